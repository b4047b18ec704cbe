#!/bin/bash
# Round 4 batch Q: ZeRO-2 at emulated N = 8 / 2 with the embedding folded into the last block bucket (DLTB_SOLO_TAIL=0:
# one collective less per micro-step) vs its own bucket (default 1); 2 interleaved rounds.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4q
for r in 1 2; do
  for n in 8 2; do
    for v in 1 0; do
      DLTB_SOLO_TAIL=$v timeout -k 10 200 python bench.py --emulate $n --steps 24 --warmup 8 --graphs off \
        > gpurun_out/r4q/e${n}_t${v}_$r.log 2>&1 || { tail -20 gpurun_out/r4q/e${n}_t${v}_$r.log; exit 1; }
      tail -n 1 gpurun_out/r4q/e${n}_t${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=$n solo_tail=$v r$r', round(d['ms_per_step'],3), {k: round(v,3) for k,v in (d.get('phase_ms') or {}).items()})"
    done
  done
done
