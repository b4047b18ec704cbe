#!/usr/bin/env bash
# Closing evidence after the in-step hipBLASLt picks and the DDP sharded-optimizer option: GPU suite, smoke, bench x3, AdamW bandwidth, steady-state kernel profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6x
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6x/gpu_tests.log 2>&1 \
  || { tail -30 gpurun_out/r6x/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r6x/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6x/smoke.log 2>&1 || { tail -20 gpurun_out/r6x/smoke.log; exit 1; }
tail -1 gpurun_out/r6x/smoke.log
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r6x/bench_$i.log 2>&1 || exit 1
done
for f in gpurun_out/r6x/bench_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
timeout -k 10 120 python scripts/bench_adamw.py > gpurun_out/r6x/adamw.log 2>&1 || { tail -5 gpurun_out/r6x/adamw.log; exit 1; }
tail -3 gpurun_out/r6x/adamw.log
bash scripts/rocprof.sh gpurun_out/r6x/prof_steady > gpurun_out/r6x/rocprof.log 2>&1 || { tail -20 gpurun_out/r6x/rocprof.log; exit 1; }
head -34 gpurun_out/r6x/prof_steady/summary_steady.txt
