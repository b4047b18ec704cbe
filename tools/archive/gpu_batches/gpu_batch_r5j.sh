#!/usr/bin/env bash
# gemm_rsf ablations + D3; AdamW path A/B and its GPU tests
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5j
export HSA_ENABLE_IPC_MODE_LEGACY=0
CFGS=43 REPS=3 timeout -k 10 200 python scripts/debug_gemm_rs.py > gpurun_out/r5j/debug.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 4 --cfgs 35,38,39,40,41,42,43 --only fc1.fwd,fc2.dgrad,qkv.fwd > gpurun_out/r5j/abl.txt 2>&1 || exit 1
for v in "" "DLTB_ADAM_T128=1" "DLTB_ADAM_WIDE=1" "" "DLTB_ADAM_T128=1"; do
  env $v timeout -k 10 120 python scripts/bench_adamw.py >> gpurun_out/r5j/adamw.txt 2>&1 || exit 1
done
DLTB_ADAM_T128=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k adamw > gpurun_out/r5j/adam_tests.txt 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k adamw >> gpurun_out/r5j/adam_tests.txt 2>&1
