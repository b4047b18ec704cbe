#!/usr/bin/env bash
# A/B of a kernel variant built with `python csrc/build.py --tag TAG [-D ...]` against the release
# extension: alternating bench.py runs on one box (DLTB_EXT_PATH selects the variant).
#   scripts/ab/ab_ext.sh TAG [ROUNDS] [bench.py flags...]
set -euo pipefail
cd "$(dirname "$0")/../.."
TAG=$1; ROUNDS=${2:-3}; shift 2 || shift $#
SO=$(ls build/$TAG/_C*.so)
mkdir -p gpurun_out
for r in $(seq "$ROUNDS"); do
  for v in base "$TAG"; do
    if [ "$v" = base ]; then E=""; else E="$SO"; fi
    DLTB_EXT_PATH=$E timeout -k 10 200 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/abx_${v}_$r.log 2>&1
    echo "$v run $r: $(tail -n 1 gpurun_out/abx_${v}_$r.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
