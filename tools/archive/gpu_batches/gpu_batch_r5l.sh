#!/usr/bin/env bash
# in-step A/B of the own kernel on the N = 1024 products; kernel profiles of both arms
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5l
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=configs/gemm_rs/ab_rsf_n1024.csv
for i in 1 2 3; do
  DLTB_OWN_GEMM=0 timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r5l/bench_off_$i.log 2>&1 || exit 1
  DLTB_OWN_GEMM_TABLE=$T timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r5l/bench_on_$i.log 2>&1 || exit 1
done
DLTB_OWN_GEMM=0 bash scripts/rocprof.sh gpurun_out/r5l/prof_off > gpurun_out/r5l/prof_off.log 2>&1 || exit 1
DLTB_OWN_GEMM_TABLE=$PWD/$T bash scripts/rocprof.sh gpurun_out/r5l/prof_on > gpurun_out/r5l/prof_on.log 2>&1
