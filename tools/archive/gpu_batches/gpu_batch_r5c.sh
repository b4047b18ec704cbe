#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5c
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python scripts/debug_gemm_rs.py 2>&1 | tee gpurun_out/r5c/debug.txt
SHAPE=2048,1024,4096 CFGS=1,2 bash scripts/pmc_gemm_rs.sh gpurun_out/r5c/pmc_fc2 2>&1 | tee gpurun_out/r5c/pmc_fc2.txt
