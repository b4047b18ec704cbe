#!/bin/bash
# Round 4 batch J: world-8 host-staged equivalence on one GPU (8 ranks share cuda:0).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests/test_multirank_gpu.py -x -v -s --timeout 960 --timeout-method thread \
  -k "world8" -p no:cacheprovider > gpurun_out/r4j_ws8.log 2>&1; rc=$?
grep -E "multirank|passed|failed|Error" gpurun_out/r4j_ws8.log | tail -8
exit $rc
