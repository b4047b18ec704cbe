#!/usr/bin/env bash
# pipelined gemm_rsp: correctness then timing vs hipBLASLt and the 2-buffer kernel
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5h
export HSA_ENABLE_IPC_MODE_LEGACY=0
REPS=5 timeout -k 10 300 python scripts/debug_gemm_rs.py 2>&1 | grep -v "^   " | tee gpurun_out/r5h/debug.txt
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 1,4 --cfgs 1,2,4,5,26,27,28,29,30,31 2>&1 | tee gpurun_out/r5h/rs_warm.txt
