#!/usr/bin/env bash
# gemm_rs debug + direct-operand variants + PMC, AdamW 16-byte path A/B, AdamW / FlatAdamW numerics
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5d
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python scripts/debug_gemm_rs.py 2>&1 | tee gpurun_out/r5d/debug.txt
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 4 --cfgs 0,1,3,5,8,9,10,11,12 2>&1 | tee gpurun_out/r5d/rs_warm.txt
for r in 1 2; do
  timeout -k 10 120 python scripts/bench_adamw.py 2>&1 | tail -1
  DLTB_ADAM_NARROW=1 timeout -k 10 120 python scripts/bench_adamw.py 2>&1 | tail -1
done | tee gpurun_out/r5d/adamw.txt
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "adamw or sumsq" 2>&1 | tail -3
SHAPE=2048,1024,4096 CFGS=1,9 bash scripts/pmc_gemm_rs.sh gpurun_out/r5d/pmc_fc2 2>&1 | tee gpurun_out/r5d/pmc_fc2.txt
