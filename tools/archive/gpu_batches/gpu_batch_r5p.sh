#!/usr/bin/env bash
# ddp_bf16 phase breakdown (world 1 vs emulated N = 8 variants), then the FSDP rows of the predicted table
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
STRAT=ddp BASE="--dtype bf16" bash scripts/emu_phases.sh > gpurun_out/emu_phases_ddp_bf16_r5.txt 2>&1 || { cat gpurun_out/emu_phases_ddp_bf16_r5.txt; exit 1; }
cat gpurun_out/emu_phases_ddp_bf16_r5.txt
SUFFIX=_b STRATS="fsdp_bf16_sgo fsdp_sgo" bash scripts/gpu_batch_r5o.sh
