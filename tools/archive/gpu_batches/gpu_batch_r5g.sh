#!/usr/bin/env bash
# gemm_rs with the coalesced LDS epilogue: correctness (co-resident grids), ablations, all products
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5g
export HSA_ENABLE_IPC_MODE_LEGACY=0
REPS=3 timeout -k 10 300 python scripts/debug_gemm_rs.py 2>&1 | grep -v "^   " | tee gpurun_out/r5g/debug.txt
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 4 --cfgs 4,16,17,18,19,24 --only fc1.fwd 2>&1 | tee gpurun_out/r5g/abl_c4.txt
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 4 --cfgs 1,20,21,22,23,25 --only fc2.fwd 2>&1 | tee gpurun_out/r5g/abl_c1.txt
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 1,4 --cfgs 0,1,2,4,5,6,8,10,11 2>&1 | tee gpurun_out/r5g/rs_warm.txt
