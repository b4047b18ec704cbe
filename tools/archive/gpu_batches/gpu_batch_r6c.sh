#!/usr/bin/env bash
# same-box kernel traces: shipped table vs the dGELU-epilogue table
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6c
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/rocprof.sh gpurun_out/r6c/prof_ship > gpurun_out/r6c/prof_ship.log 2>&1 || exit 1
DLTB_OWN_GEMM_TABLE=$PWD/configs/gemm_rs/ab_dgelu62.csv bash scripts/rocprof.sh gpurun_out/r6c/prof_d62 > gpurun_out/r6c/prof_d62.log 2>&1
