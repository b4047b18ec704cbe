#!/usr/bin/env bash
# dGELU epilogue: numerics, model equivalence with the table on, interleaved in-step A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6a
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_rs_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6a/tests.log 2>&1 || { tail -30 gpurun_out/r6a/tests.log; exit 1; }
tail -1 gpurun_out/r6a/tests.log
DLTB_OWN_GEMM_TABLE=configs/gemm_rs/ab_dgelu35.csv timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6a/model_tests.log 2>&1 || { tail -30 gpurun_out/r6a/model_tests.log; exit 1; }
tail -1 gpurun_out/r6a/model_tests.log
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r6a/bench_ship_$i.log 2>&1 || exit 1
  DLTB_OWN_GEMM_TABLE=configs/gemm_rs/ab_dgelu35.csv timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r6a/bench_d35_$i.log 2>&1 || exit 1
  DLTB_OWN_GEMM_TABLE=configs/gemm_rs/ab_dgelu62.csv timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r6a/bench_d62_$i.log 2>&1 || exit 1
done
for f in gpurun_out/r6a/bench_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
