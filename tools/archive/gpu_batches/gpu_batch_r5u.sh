#!/usr/bin/env bash
# in-step kernel profile with every per-layer product on the own kernel (per-product in-step times)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5u
export HSA_ENABLE_IPC_MODE_LEGACY=0
DLTB_OWN_GEMM_TABLE=$PWD/configs/gemm_rs/ab_rsf_all.csv bash scripts/rocprof.sh gpurun_out/r5u/prof_all > gpurun_out/r5u/prof_all.log 2>&1 || exit 1
head -40 gpurun_out/r5u/prof_all/summary_steady.txt
