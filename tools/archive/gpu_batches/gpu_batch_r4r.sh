#!/bin/bash
# Round 4 batch R: ZeRO-2 emulated N = 8 / 2 with 4-block (64 MiB -> 101 MB) vs 8-block (128 MiB -> 202 MB) buckets.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4r
for r in 1 2; do
  for n in 8 2; do
    for v in 64 128; do
      timeout -k 10 200 python bench.py --emulate $n --steps 24 --warmup 8 --graphs off --bucket-mb $v \
        > gpurun_out/r4r/e${n}_t${v}_$r.log 2>&1 || { tail -20 gpurun_out/r4r/e${n}_t${v}_$r.log; exit 1; }
      tail -n 1 gpurun_out/r4r/e${n}_t${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=$n bucket_mb=$v r$r', round(d['ms_per_step'],3), {k: round(v,3) for k,v in (d.get('phase_ms') or {}).items()})"
    done
  done
done
