#!/bin/bash
# Round 4 batch N: sharded engines' tied-table gather first (DLTB_AG_TIED_FIRST 1 vs 0), emulated N = 8 ZeRO-3 and FSDP
# (predictions), 2 interleaved rounds; then the world-2 / -8 host-staged equivalence tests.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4n
for r in 1 2; do
  for s in zero3 fsdp; do
    for v in 1 0; do
      DLTB_AG_TIED_FIRST=$v timeout -k 10 200 python bench.py --strategy $s --emulate 8 --steps 24 --warmup 8 --graphs off \
        > gpurun_out/r4n/${s}_v${v}_$r.log 2>&1 || { tail -20 gpurun_out/r4n/${s}_v${v}_$r.log; exit 1; }
      tail -n 1 gpurun_out/r4n/${s}_v${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$s N=8 tied_first=$v r$r', round(d['ms_per_step'],3), {k: round(v,3) for k,v in (d.get('phase_ms') or {}).items()})"
    done
  done
done
timeout -k 10 1000 python -u -m pytest tests/test_multirank_gpu.py -x -q --timeout 960 --timeout-method thread \
  -k "world2_host_staged or world8" -p no:cacheprovider > gpurun_out/r4n/mr.log 2>&1 || { tail -30 gpurun_out/r4n/mr.log; exit 1; }
tail -1 gpurun_out/r4n/mr.log
