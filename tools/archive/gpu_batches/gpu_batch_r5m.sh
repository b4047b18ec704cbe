#!/usr/bin/env bash
# cfg 34 family: ablations and variants on the N = 1024 products
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5m
export HSA_ENABLE_IPC_MODE_LEGACY=0
CFGS=49,50,51 REPS=3 timeout -k 10 200 python scripts/debug_gemm_rs.py > gpurun_out/r5m/debug.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 1,4 --cfgs 34,49,50,51 --only out.fwd,fc2.fwd,fc1.dgrad,out.dgrad,qkv.dgrad > gpurun_out/r5m/var.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 4 --cfgs 34,44,45,46,47,48 --only fc2.fwd,out.dgrad > gpurun_out/r5m/abl.txt 2>&1
