#!/usr/bin/env bash
# gemm_rs ablations (timing only: the ablated configs compute garbage) + PMC of cfg 4 / cfg 1 vs hipBLASLt
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5f
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 4 --cfgs 4,16,17,18,19 --only fc1.fwd 2>&1 | tee gpurun_out/r5f/abl_c4.txt
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 4 --cfgs 1,20,21,22,23 --only fc2.fwd 2>&1 | tee gpurun_out/r5f/abl_c1.txt
SHAPE=2048,4096,1024 CFGS=4 bash scripts/pmc_gemm_rs.sh gpurun_out/r5f/pmc_fc1 2>&1 | tee gpurun_out/r5f/pmc_fc1.txt
