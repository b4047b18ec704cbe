#!/usr/bin/env bash
# Lockstep test of the forward's key splits: KS=3 (one 12-wave workgroup per CU, splits share
# the per-tile barrier) vs KS=1 (4-wave workgroups) on 1 and 3 micro-batches (768 query blocks:
# three independent KS=1 workgroups per CU).
set -e
SO=$(ls build/fks1/_C*.so)
for r in 1 2; do
  echo "KS3:"; timeout -k 10 120 python scripts/bench_attn.py --iters 30 --shapes tinygpt_a,tinygpt_a_b3 2>&1 | grep " fwd"
  echo "KS1:"; DLTB_EXT_PATH=$SO timeout -k 10 120 python scripts/bench_attn.py --iters 30 --shapes tinygpt_a,tinygpt_a_b3 2>&1 | grep " fwd"
done
