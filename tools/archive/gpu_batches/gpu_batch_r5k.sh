#!/usr/bin/env bash
# fp32-image epilogue + bias prefetch timing; own-GEMM in-step check and interleaved bench A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5k
export HSA_ENABLE_IPC_MODE_LEGACY=0
REPS=3 timeout -k 10 200 python scripts/debug_gemm_rs.py > gpurun_out/r5k/debug.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 1,4 --cfgs 34,35,36 > gpurun_out/r5k/rs_warm.txt 2>&1 || exit 1
DLTB_OWN_GEMM_TABLE=configs/gemm_rs/ab_rsf_all.csv timeout -k 10 200 python scripts/own_gemm_check.py > gpurun_out/r5k/check.txt 2>&1 || exit 1
for i in 1 2 3; do
  DLTB_OWN_GEMM=0 timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r5k/bench_off_$i.log 2>&1 || exit 1
  DLTB_OWN_GEMM_TABLE=configs/gemm_rs/ab_rsf_all.csv timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r5k/bench_on_$i.log 2>&1 || exit 1
done
