#!/usr/bin/env bash
# One GPU-box check of the current tree: the GPU test suite, the 1-GPU flagship bench (twice),
# a steady-state rocprofv3 kernel profile and the attention PMC passes.  Outputs under gpurun_out/.
set -eo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
tail -2 gpurun_out/gpu_tests.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$r.log 2>&1
  tail -n 1 gpurun_out/bench_$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' '; echo
done
bash scripts/rocprof.sh gpurun_out/prof_steady > gpurun_out/rocprof.log 2>&1
head -20 gpurun_out/prof_steady/summary_steady.txt
if [ "${PMC:-0}" = 1 ]; then
  bash scripts/pmc_attn.sh gpurun_out/pmc_attn > gpurun_out/pmc_attn.txt 2>&1
  grep -A1 "attn_fwd\|attn_bwd_dq\|attn_bwd_dkdv" gpurun_out/pmc_attn.txt | head -30
fi
