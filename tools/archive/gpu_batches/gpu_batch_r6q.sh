#!/usr/bin/env bash
# ddp_bf16_zero1 emulated rows with the solo-tail layout (r6p)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6q; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python scripts/emulated_scaling.py --strategies ddp_bf16 ddp_bf16_zero1 --out $O/emulated.txt > $O/emu.log 2>&1 || { tail -20 $O/emu.log; exit 1; }
cat $O/emulated.txt
