#!/usr/bin/env bash
# PMC counters: shipped own kernel (cfg 34) vs hipBLASLt on fc2.fwd (2048 x 1024 x 4096) and out.fwd (x 1024)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6f
export HSA_ENABLE_IPC_MODE_LEGACY=0
SHAPE=2048,1024,4096 CFGS=34 bash scripts/pmc_gemm_rs.sh gpurun_out/r6f/fc2 > gpurun_out/r6f/fc2.txt 2>&1 || { cat gpurun_out/r6f/fc2.txt; exit 1; }
SHAPE=2048,1024,1024 CFGS=34 bash scripts/pmc_gemm_rs.sh gpurun_out/r6f/out > gpurun_out/r6f/out.txt 2>&1
cat gpurun_out/r6f/fc2.txt
