#!/usr/bin/env bash
# Round-5 closing evidence: GPU suite, smoke, bench twice, out-proj cfg 69 in-step A/B, steady-state kernel profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5y
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5y/gpu_tests.log 2>&1 \
  || { tail -30 gpurun_out/r5y/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5y/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5y/smoke.log 2>&1 || { tail -20 gpurun_out/r5y/smoke.log; exit 1; }
tail -1 gpurun_out/r5y/smoke.log
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r5y/bench_ship_$i.log 2>&1 || exit 1
  DLTB_OWN_GEMM_TABLE=configs/gemm_rs/ab_rsf_out69.csv timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r5y/bench_out69_$i.log 2>&1 || exit 1
done
for f in gpurun_out/r5y/bench_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
bash scripts/rocprof.sh gpurun_out/r5y/prof_steady > gpurun_out/r5y/rocprof.log 2>&1 || { tail -20 gpurun_out/r5y/rocprof.log; exit 1; }
head -34 gpurun_out/r5y/prof_steady/summary_steady.txt
