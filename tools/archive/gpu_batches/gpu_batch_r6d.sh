#!/usr/bin/env bash
# Mistral-7B shape (BASELINE config #5), ZeRO-3, seq 4096, 1 GPU: round-5 tree
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6d
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python bench.py --strategy zero3 --tier M7B --seq-len 4096 --steps 8 --warmup 8 > gpurun_out/r6d/m7b_1gpu.log 2>&1 || { tail -20 gpurun_out/r6d/m7b_1gpu.log; exit 1; }
tail -n 1 gpurun_out/r6d/m7b_1gpu.log
