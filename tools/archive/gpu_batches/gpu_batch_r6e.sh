#!/usr/bin/env bash
# in-step A/B of own-kernel config variants on the N = 1024 products
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6e
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r6e/bench_ship_$i.log 2>&1 || exit 1
  DLTB_OWN_GEMM_TABLE=configs/gemm_rs/ab_rsf_out49.csv timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r6e/bench_out49_$i.log 2>&1 || exit 1
  DLTB_OWN_GEMM_TABLE=configs/gemm_rs/ab_rsf_q50.csv timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r6e/bench_q50_$i.log 2>&1 || exit 1
done
for f in gpurun_out/r6e/bench_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
