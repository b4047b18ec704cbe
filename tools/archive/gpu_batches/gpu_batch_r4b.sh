#!/usr/bin/env bash
# Round-4 GPU batch B: the PREDICTED scaling table (emulated fabric) for every strategy incl. the
# bf16 DDP / FSDP rows of BASELINE configs #2 / #3.  Writes gpurun_out/emulated_scaling_r4.{txt,jsonl}.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rm -f gpurun_out/emulated_scaling_r4.jsonl
timeout -k 10 1100 python scripts/emulated_scaling.py --out gpurun_out/emulated_scaling_r4.txt \
    --strategies ${STRATS:-zero2 zero3 fsdp fsdp_root ddp ddp_bf16 fsdp_bf16} ${EXTRA_ARGS:-}
