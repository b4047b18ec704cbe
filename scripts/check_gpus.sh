#!/usr/bin/env bash
# Node readiness check (replaces the reference's K8s GPU checker, scripts/check_cluster_gpus.sh):
# visible MI355X GPUs, HBM, xGMI topology, RCCL / torch versions and the built HIP extension.
set -uo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
echo "== ROCm tools"
command -v rocm-smi >/dev/null && rocm-smi --showproductname --showmeminfo vram 2>/dev/null | head -40
command -v rocm-smi >/dev/null && { echo "== xGMI topology"; rocm-smi --showtopotype 2>/dev/null | head -20; }
echo "== torch / RCCL"
python3 - <<'PY'
import torch
print("torch", torch.__version__, "hip", torch.version.hip)
n = torch.cuda.device_count()
print("visible GPUs:", n)
for i in range(n):
    p = torch.cuda.get_device_properties(i)
    print(f"  [{i}] {p.name} {getattr(p, 'gcnArchName', '')} CUs={p.multi_processor_count} HBM={p.total_memory/1e9:.0f} GB")
try:
    print("RCCL", torch.cuda.nccl.version())
except Exception as e:
    print("RCCL version unavailable:", e)
PY
echo "== dltb extension"
( cd "$ROOT" && python3 -c "import dltb; from dltb.ops._ext import available, so_path; print('dltb._C', 'OK' if available() else 'MISSING', so_path())" )
if [[ "${HSA_ENABLE_IPC_MODE_LEGACY:-}" != "0" ]]; then
  echo "WARNING: export HSA_ENABLE_IPC_MODE_LEGACY=0 for multi-process RCCL on this platform"
fi
