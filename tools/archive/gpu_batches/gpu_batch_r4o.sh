#!/bin/bash
# Round 4 batch O: predicted ZeRO-2 / ZeRO-3 rows of the final round-4 tree (emulated fabric, one MI355X plays rank 0).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1100 python -u scripts/emulated_scaling.py --strategies ${STRATS:-zero2 zero3} --out gpurun_out/emulated_scaling_r4_final${SUFFIX:-}.txt \
  > gpurun_out/emulated_scaling_r4_final${SUFFIX:-}.log 2>&1 || { tail -30 gpurun_out/emulated_scaling_r4_final${SUFFIX:-}.log; exit 1; }
cat gpurun_out/emulated_scaling_r4_final${SUFFIX:-}.txt
