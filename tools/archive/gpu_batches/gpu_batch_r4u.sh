#!/bin/bash
# Round 4 batch U: ZeRO-2 emulated N = 8 / 2, early bucket of 8 blocks (DLTB_EARLY_MULT=2) vs 12 (3).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4u
for r in 1 2; do
  for n in 8 2; do
    for v in 2 3; do
      DLTB_EARLY_MULT=$v timeout -k 10 200 python bench.py --emulate $n --steps 24 --warmup 8 --graphs off   \
        > gpurun_out/r4u/e${n}_t${v}_$r.log 2>&1 || { tail -20 gpurun_out/r4u/e${n}_t${v}_$r.log; exit 1; }
      tail -n 1 gpurun_out/r4u/e${n}_t${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=$n early_mult=$v r$r', round(d['ms_per_step'],3), {k: round(v,3) for k,v in (d.get('phase_ms') or {}).items()})"
    done
  done
done
