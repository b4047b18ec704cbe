#!/usr/bin/env bash
# PMC counters of gemm_rs against hipBLASLt on one product shape (SHAPE=M,N,K, CFGS=...), one rocprofv3 pass
# per counter group.   ./scripts/pmc_gemm_rs.sh OUTDIR
set -uo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${1:-$ROOT/gpurun_out/pmc_gemm_rs}"
mkdir -p "$OUT"
OUT="$(cd "$OUT" && pwd)"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name="$1"; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/$name" -o run -- \
    python3 "$ROOT/scripts/gemm_rs_probe.py" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS && \
pass sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_LDS && \
pass tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT && \
python3 "$ROOT/scripts/pmc_table.py" "$OUT/sq1" "$OUT/sq2" "$OUT/tcc"
