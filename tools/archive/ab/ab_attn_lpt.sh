#!/usr/bin/env bash
# Causal forward / dQ grid order A/B at the M7B shape: release (XCD-remapped sweeps) vs build/lpt
# (heaviest query blocks first over the whole grid, DLTB_ATTN_LPT=1)
set -o pipefail
cd "$(dirname "$0")/../.."
SO=$(ls build/lpt/_C*.so)
for r in 1 2 3; do
  for v in base lpt; do
    if [ $v = lpt ]; then E=$SO; else E=""; fi
    DLTB_EXT_PATH=$E timeout -k 5 120 python scripts/bench_attn.py --shapes m7b --iters 20 > gpurun_out/abl_${v}_$r.log 2>&1 || exit 1
    echo "$v r$r: $(grep -E 'fwd|dq|total' gpurun_out/abl_${v}_$r.log | tr -s ' ' | tr '\n' ' ')"
  done
done
