#!/usr/bin/env bash
# fenced kernel at 8 waves per workgroup (2 per SIMD)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5w
export HSA_ENABLE_IPC_MODE_LEGACY=0
CFGS=62,63,64,65,66 REPS=3 timeout -k 10 200 python scripts/debug_gemm_rs.py > gpurun_out/r5w/debug.txt 2>&1 || { cat gpurun_out/r5w/debug.txt; exit 1; }
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 1,4 --cfgs 34,35,36,62,63,64,65,66 > gpurun_out/r5w/rs_warm.txt 2>&1
