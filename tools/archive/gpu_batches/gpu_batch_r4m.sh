#!/bin/bash
# Round 4 batch M: deferred ZeRO-2 update A/B (env VAR, default 1 vs 0): the tied table bucket first / the per-bucket AdamW + all-gather pipeline;
# emulated N = 2 and N = 8 (predictions), 2 interleaved rounds; then the world-2 / -8 host-staged equivalence tests.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
VAR=${VAR:-DLTB_AG_TIED_FIRST}
mkdir -p gpurun_out/r4m
for r in 1 2; do
  for n in 2 8; do
    for v in 1 0; do
      env $VAR=$v timeout -k 10 200 python bench.py --emulate $n --steps 24 --warmup 8 --graphs off \
        > gpurun_out/r4m/e${n}_v${v}_$r.log 2>&1 || { tail -20 gpurun_out/r4m/e${n}_v${v}_$r.log; exit 1; }
      tail -n 1 gpurun_out/r4m/e${n}_v${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=$n $VAR=$v r$r', round(d['ms_per_step'],3), {k: round(v,3) for k,v in (d.get('phase_ms') or {}).items()})"
    done
  done
done
timeout -k 10 1000 python -u -m pytest tests/test_multirank_gpu.py -x -q --timeout 960 --timeout-method thread \
  -k "world2_host_staged or world8" -p no:cacheprovider > gpurun_out/r4m/mr.log 2>&1 || { tail -30 gpurun_out/r4m/mr.log; exit 1; }
tail -1 gpurun_out/r4m/mr.log
