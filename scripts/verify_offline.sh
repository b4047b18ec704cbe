#!/usr/bin/env bash
# Offline readiness check of the dltb image (reference: scripts/verify_offline.sh, its only "test").
# Runs without a GPU and without network: every check executes inside `docker run --network none`
# (or directly on this host with --local) and verifies
#   1. the Python stack imports (torch-ROCm, numpy, pandas, matplotlib, yaml) with no download,
#   2. the in-tree HIP extension is present and built for gfx950 (code object check, no GPU needed),
#   3. TinyGPT Tier A / Tier B and the Mistral-7B shape instantiate on the CPU with the expected
#      parameter counts (236.41M / 1,681.2M / 7.24B - the latter on the meta device),
#   4. the synthetic dataset yields [batch, seq] int64 token blocks,
#   5. one CPU training step of a tiny model runs through an engine (gloo-free, world size 1).
# Usage: scripts/verify_offline.sh [IMAGE]      or      scripts/verify_offline.sh --local
set -euo pipefail
IMAGE="${1:-${IMAGE:-dltb:mi355x}}"
ROOT="$(cd "$(dirname "$0")/.." && pwd)"

run() {
  if [[ "$IMAGE" == "--local" ]]; then
    (cd "$ROOT" && env HF_HUB_OFFLINE=1 TRANSFORMERS_OFFLINE=1 python3 -c "$1")   # inherits VERIFY_ALLOW_NO_EXT
  else
    docker run --rm --network none -e HF_HUB_OFFLINE=1 -e TRANSFORMERS_OFFLINE=1 -w /workspace "$IMAGE" python3 -c "$1"
  fi
}

echo "== 1. imports"
run 'import torch, numpy, pandas, yaml, matplotlib; print("torch", torch.__version__, "hip", torch.version.hip)'

echo "== 2. HIP extension (gfx950 code object)"
run '
import dltb
from dltb.ops._ext import so_path
import os, sys
p = so_path()
if not p and os.environ.get("VERIFY_ALLOW_NO_EXT") == "1":
    print("dltb._C not built here (allowed: VERIFY_ALLOW_NO_EXT=1)"); sys.exit(0)
assert p, "dltb._C is not built"
blob = open(p, "rb").read()
assert b"amdgcn-amd-amdhsa--gfx950" in blob, "extension carries no gfx950 code object"
print(p, "-> gfx950 code object present")
'

echo "== 3. models instantiate (CPU / meta)"
run '
import torch, dltb
from dltb.models import build_model, get_model_config
for tier, want in (("A", 236.41e6), ("B", 1681.2e6)):
    with torch.device("meta"):
        m = build_model(get_model_config(tier, 2048))
    n = sum(p.numel() for p in m.parameters())
    print(f"TinyGPT tier {tier}: {n/1e6:.2f}M params")
    assert abs(n - want) / want < 1e-3
with torch.device("meta"):
    m = build_model(get_model_config("M7B", 4096))
print(f"Mistral-7B shape: {sum(p.numel() for p in m.parameters())/1e9:.2f}B params")
'

echo "== 4. synthetic dataset"
run '
import dltb
from dltb.data import SyntheticDataset
ds = SyntheticDataset(32000, 2048, size=8, seed=42)
x = ds[0]
print("sample", tuple(x.shape), x.dtype)
assert x.shape == (2048,) and str(x.dtype) == "torch.int64"
'

echo "== 5. one CPU training step"
run '
import torch, dltb
from dltb.models import build_model, get_model_config
from dltb.parallel import engine_config, make_engine
cfg = get_model_config("tiny", 32)
m = build_model(cfg)
eng = make_engine(m, engine_config("zero2", grad_accum=1), "cpu")
idx = torch.randint(0, cfg.vocab_size, (2, 32))
loss = eng(idx, idx)[1]; eng.backward(loss); eng.step()
print("loss", loss.item())
'
echo "OFFLINE VERIFICATION PASSED"
