#!/usr/bin/env bash
# World-1 batched dW on a side stream beside the dX chain (DLTB_WGRAD_SIDE): numerics + bench A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6i
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_wgrad_side_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6i/tests.log 2>&1 || { tail -30 gpurun_out/r6i/tests.log; exit 1; }
tail -1 gpurun_out/r6i/tests.log
for i in 1 2; do
  for v in 0 2 4 8; do
    DLTB_WGRAD_SIDE=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r6i/b_${v}_$i.log 2>&1 || exit 1
    echo "side=$v $i $(tail -n 1 gpurun_out/r6i/b_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3))")"
  done
done
