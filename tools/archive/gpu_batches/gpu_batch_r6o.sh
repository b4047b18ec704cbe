#!/usr/bin/env bash
# DDP + sharded optimizer state (--ddp-shard-optimizer, ZeroRedundancyOptimizer semantics) on the emulated fabric
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6o; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python scripts/emulated_scaling.py --strategies ddp_bf16 ddp_bf16_zero1 --out $O/emulated.txt > $O/emu.log 2>&1 || { tail -20 $O/emu.log; exit 1; }
cat $O/emulated.txt
STRAT=ddp BASE="--dtype bf16 --ddp-shard-optimizer" bash scripts/emu_phases.sh > $O/phases.txt 2>&1; cat $O/phases.txt
