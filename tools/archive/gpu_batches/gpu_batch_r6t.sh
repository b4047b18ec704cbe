#!/usr/bin/env bash
# Final-tree emulated scaling rows, part $1 (A: the reference-precision strategies, B: bf16 configs #2 / #3 + options)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6t; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "$1" = A ]; then S="zero2 zero3 fsdp fsdp_sgo fsdp_root ddp"; else S="ddp_bf16 ddp_bf16_zero1 fsdp_bf16 fsdp_bf16_sgo"; fi
timeout -k 10 1100 python scripts/emulated_scaling.py --strategies $S --out $O/emulated_$1.txt > $O/emu_$1.log 2>&1 || { tail -20 $O/emu_$1.log; exit 1; }
cat $O/emulated_$1.txt
