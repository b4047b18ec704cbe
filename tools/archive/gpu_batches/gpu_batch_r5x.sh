#!/usr/bin/env bash
# 8-wave depth variants; in-step A/B of the 8-wave big-N kernels (+ kernel trace of that arm)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5x
export HSA_ENABLE_IPC_MODE_LEGACY=0
CFGS=67,68,69 REPS=3 timeout -k 10 200 python scripts/debug_gemm_rs.py > gpurun_out/r5x/debug.txt 2>&1 || { cat gpurun_out/r5x/debug.txt; exit 1; }
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 1,4 --cfgs 62,64,65,67,68,69 > gpurun_out/r5x/rs_warm.txt 2>&1 || exit 1
T=configs/gemm_rs/ab_rsf_big8.csv
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r5x/bench_ship_$i.log 2>&1 || exit 1
  DLTB_OWN_GEMM_TABLE=$T timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r5x/bench_big8_$i.log 2>&1 || exit 1
done
DLTB_OWN_GEMM_TABLE=$PWD/$T bash scripts/rocprof.sh gpurun_out/r5x/prof_big8 > gpurun_out/r5x/prof_big8.log 2>&1 || exit 1
bash scripts/rocprof.sh gpurun_out/r5x/prof_ship > gpurun_out/r5x/prof_ship.log 2>&1
