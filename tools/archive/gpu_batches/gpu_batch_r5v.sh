#!/usr/bin/env bash
# fenced kernels with the fragment register sets kept apart (no read into a register an in-flight MFMA reads)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5v
export HSA_ENABLE_IPC_MODE_LEGACY=0
CFGS=59,60,61 REPS=3 timeout -k 10 200 python scripts/debug_gemm_rs.py > gpurun_out/r5v/debug.txt 2>&1 || { cat gpurun_out/r5v/debug.txt; exit 1; }
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 1,4 --cfgs 34,35,36,59,60,61 > gpurun_out/r5v/rs_warm.txt 2>&1
