#!/usr/bin/env bash
# A/B of functional.wgrad_operands (transposed K-contiguous operand for large weight gradients) on
# the Mistral-7B-shape ZeRO-3 bench: "off" patches the gain model to zero in-process.
set -euo pipefail
cd "$(dirname "$0")/../.."
ARGS="--tier M7B --seq-len 4096 --strategy zero3 --steps 8 --warmup 4"
for r in 1 2; do
  for mode in off on; do
    G=$([ "$mode" = off ] && echo 0.0 || echo 0.15)
    timeout -k 10 250 python -c "import sys; sys.argv=['bench.py'] + '$ARGS'.split(); sys.path.insert(0, '.')
import dltb.ops.functional as F; F._WGRAD_GAIN = $G
import runpy; runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/ab_wt_${mode}_$r.log 2>&1
    echo "$mode run $r: $(tail -n 1 gpurun_out/ab_wt_${mode}_$r.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
