#!/usr/bin/env bash
# Round-5 GEMM iteration: gemm_rs (register-staged NT GEMM) vs hipBLASLt on the TinyGPT-A per-layer products.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5b
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 1,4 2>&1 | tee gpurun_out/r5b/rs_warm.txt
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 20 --gm 4 --cold 2>&1 | tee gpurun_out/r5b/rs_cold.txt
