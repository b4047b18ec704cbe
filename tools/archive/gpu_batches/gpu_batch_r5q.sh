#!/usr/bin/env bash
# DDP pipeline with the token rows applied last: ddp_bf16 phases + predicted rows
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
STRAT=ddp BASE="--dtype bf16" bash scripts/emu_phases.sh > gpurun_out/emu_phases_ddp_bf16_r5b.txt 2>&1 || { cat gpurun_out/emu_phases_ddp_bf16_r5b.txt; exit 1; }
cat gpurun_out/emu_phases_ddp_bf16_r5b.txt
SUFFIX=_c STRATS="ddp_bf16 ddp" bash scripts/gpu_batch_r5o.sh
