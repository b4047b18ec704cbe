#!/usr/bin/env bash
# Kernel-level comparison of the world-1 eager step and the emulated N-rank step (fabric made
# infinitely fast and no traffic stream (PASSES=0), so only the N-rank code path differs): rocprofv3 steady-state summaries under
# gpurun_out/prof_w1_eager and gpurun_out/prof_e${N}_fast.
set -o pipefail
cd "$(dirname "$0")/.."
N="${N:-8}"; S="${STRAT:-zero2}"
bash scripts/rocprof.sh gpurun_out/prof_w1_eager --strategy $S --graphs off > gpurun_out/prof_w1_eager.log 2>&1 || exit 1
head -40 gpurun_out/prof_w1_eager/summary_steady.txt
DLTB_EMU_ALPHA_US=0 DLTB_EMU_BUS_GBPS=1e9 DLTB_EMU_HBM_PASSES=${PASSES:-0} DLTB_EMU_HOST_US=0 bash scripts/rocprof.sh gpurun_out/prof_e${N}_fast --strategy $S --emulate $N \
  > gpurun_out/prof_e${N}_fast.log 2>&1 || exit 1
head -40 gpurun_out/prof_e${N}_fast/summary_steady.txt
