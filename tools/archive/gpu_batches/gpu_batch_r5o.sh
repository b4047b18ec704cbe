#!/usr/bin/env bash
# Round-5 predicted scaling rows on the emulated fabric (one MI355X plays rank 0); STRATS / SUFFIX select the part
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/emulated_scaling_r5${SUFFIX:-}
rm -f $OUT.jsonl
timeout -k 10 1150 python -u scripts/emulated_scaling.py --strategies ${STRATS:-zero2 zero3 ddp_bf16} --out $OUT.txt > $OUT.log 2>&1 \
  || { tail -30 $OUT.log; exit 1; }
cat $OUT.txt
