#!/usr/bin/env bash
# Host enqueue vs GPU time of the eager N-rank ZeRO-2 step (emulated N=8) and the 1-GPU bench.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --strategy zero2 --emulate 8 --steps 12 --warmup 8 --host-check > gpurun_out/hc_z2_$r.log 2>&1 || exit 1
  echo "zero2 e8 r$r: $(tail -n 1 gpurun_out/hc_z2_$r.log | grep -o '"predicted_ms_per_step": [0-9.]*\|"host_over_gpu": [0-9.]*\|"host_enqueue_ms_per_step": [0-9.]*' | tr '\n' ' ')"
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/hc_w1.log 2>&1 || exit 1
echo "world 1: $(tail -n 1 gpurun_out/hc_w1.log | grep -o '"ms_per_step": [0-9.]*')"
