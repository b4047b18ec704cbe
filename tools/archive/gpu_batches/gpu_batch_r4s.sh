#!/bin/bash
# Round 4 batch S: ZeRO-2 emulated N = 8 / 2, one 8-block bucket first in the backward (DLTB_EARLY_BUCKETS=1) vs 4-block buckets.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4s
for r in 1 2; do
  for n in 8 2; do
    for v in 0 1; do
      DLTB_EARLY_BUCKETS=$v timeout -k 10 200 python bench.py --emulate $n --steps 24 --warmup 8 --graphs off   \
        > gpurun_out/r4s/e${n}_t${v}_$r.log 2>&1 || { tail -20 gpurun_out/r4s/e${n}_t${v}_$r.log; exit 1; }
      tail -n 1 gpurun_out/r4s/e${n}_t${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=$n early=$v r$r', round(d['ms_per_step'],3), {k: round(v,3) for k,v in (d.get('phase_ms') or {}).items()})"
    done
  done
done
