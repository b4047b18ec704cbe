#!/usr/bin/env bash
# fenced-schedule gemm_rsf: correctness then timing vs hipBLASLt and the pipelined kernel
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5i
export HSA_ENABLE_IPC_MODE_LEGACY=0
REPS=5 timeout -k 10 300 python scripts/debug_gemm_rs.py > gpurun_out/r5i/debug.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 1,4 --cfgs 2,28,29,32,33,34,35,36,37 > gpurun_out/r5i/rs_warm.txt 2>&1
