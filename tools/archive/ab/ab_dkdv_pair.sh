#!/usr/bin/env bash
# dK/dV key-block pairing A/B at the M7B shape: release (heaviest-first) vs build/pair (kb, nkb-1-kb on one CU)
set -o pipefail
cd "$(dirname "$0")/../.."
SO=$(ls build/pair/_C*.so)
for r in 1 2 3; do
  for v in base pair; do
    if [ $v = pair ]; then E=$SO; else E=""; fi
    DLTB_EXT_PATH=$E timeout -k 5 120 python scripts/bench_attn.py --shapes m7b --iters 20 > gpurun_out/abp_${v}_$r.log 2>&1 || exit 1
    echo "$v r$r: $(grep -E 'dkdv' gpurun_out/abp_${v}_$r.log | tr -s ' ')"
  done
done
