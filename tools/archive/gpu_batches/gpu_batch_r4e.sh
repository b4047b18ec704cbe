#!/usr/bin/env bash
# Round-4 evidence batch: steady-state rocprofv3 of the flagship (graphs, as bench.py runs it), the Mistral-7B
# ZeRO-3 1-GPU bench, Tier A at micro-batch 4, and the capability runs.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/rocprof.sh gpurun_out/prof_steady_r4 > gpurun_out/rocprof_r4.log 2>&1 || exit 1
head -32 gpurun_out/prof_steady_r4/summary_steady.txt
timeout -k 10 600 python bench.py --strategy zero3 --tier M7B --seq-len 4096 --steps 8 --warmup 8 > gpurun_out/m7b_1gpu_r4.log 2>&1 || exit 1
tail -n 1 gpurun_out/m7b_1gpu_r4.log | cut -c1-400
timeout -k 10 300 python bench.py --per-device-batch 4 --steps 12 --warmup 8 > gpurun_out/a_b4_r4.log 2>&1 || exit 1
tail -n 1 gpurun_out/a_b4_r4.log | cut -c1-300
bash scripts/capability_runs.sh
