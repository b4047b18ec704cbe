#!/usr/bin/env bash
# Interleaved scripts/bench_attn.py A/B of attention builds (csrc/build.py --tag T): base vs each tag,
# plus the attention GPU tests on the first tag.   scripts/ab/ab_attn_tags.sh ROUNDS TAG [TAG...]
set -e
mkdir -p gpurun_out
R=$1; shift
DLTB_EXT_PATH=$(ls build/$1/_C*.so) timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -x -q -k "attn or attention" --timeout 120 --timeout-method thread > gpurun_out/attn_tags_tests.log 2>&1
tail -1 gpurun_out/attn_tags_tests.log
for r in $(seq $R); do
  echo "base:"; timeout -k 10 120 python scripts/bench_attn.py --iters 50 --shapes tinygpt_a 2>&1 | grep -v amdgpu | head -3
  for t in "$@"; do
    echo "$t:"; DLTB_EXT_PATH=$(ls build/$t/_C*.so) timeout -k 10 120 python scripts/bench_attn.py --iters 50 --shapes tinygpt_a 2>&1 | grep -v amdgpu | head -3
  done
done
