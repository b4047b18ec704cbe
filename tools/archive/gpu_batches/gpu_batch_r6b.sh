#!/usr/bin/env bash
# dGELU epilogue with the aux operand prefetched at kernel start: numerics, in-step A/B, kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6b
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_rs_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6b/tests.log 2>&1 || { tail -30 gpurun_out/r6b/tests.log; exit 1; }
tail -1 gpurun_out/r6b/tests.log
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r6b/bench_ship_$i.log 2>&1 || exit 1
  DLTB_OWN_GEMM_TABLE=configs/gemm_rs/ab_dgelu62.csv timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r6b/bench_d62_$i.log 2>&1 || exit 1
done
for f in gpurun_out/r6b/bench_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
DLTB_OWN_GEMM_TABLE=$PWD/configs/gemm_rs/ab_dgelu62.csv bash scripts/rocprof.sh gpurun_out/r6b/prof_d62 > gpurun_out/r6b/prof.log 2>&1
