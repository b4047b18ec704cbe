#!/usr/bin/env bash
# gemm_rs with fragment-liveness protection: correctness under co-residency, then timings
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5e
export HSA_ENABLE_IPC_MODE_LEGACY=0
REPS=10 timeout -k 10 300 python scripts/debug_gemm_rs.py 2>&1 | tee gpurun_out/r5e/debug2.txt
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 4 --cfgs 0,1,2,4,5,8,9,10,11,12 2>&1 | tee gpurun_out/r5e/rs_warm2.txt
