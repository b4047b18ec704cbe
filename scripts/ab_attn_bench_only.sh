#!/usr/bin/env bash
# Timing-only interleaved bench_attn A/B of attention builds (no numerics: for experiment builds
# such as DLTB_ATTN_NODMA whose results are wrong by design).   scripts/ab_attn_bench_only.sh ROUNDS TAG...
set -e
R=$1; shift
for r in $(seq $R); do
  echo "base:"; timeout -k 10 120 python scripts/bench_attn.py --iters 30 --shapes tinygpt_a,m7b 2>&1 | grep " fwd\| dq\| dkdv"
  for t in "$@"; do
    echo "$t:"; DLTB_EXT_PATH=$(ls build/$t/_C*.so) timeout -k 10 120 python scripts/bench_attn.py --iters 30 --shapes tinygpt_a,m7b 2>&1 | grep " fwd\| dq\| dkdv"
  done
done
