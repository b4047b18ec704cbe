#!/usr/bin/env bash
# A/B of attention-kernel variants built by csrc/build.py --tag: numerics tests on the first
# variant, then interleaved scripts/bench_attn.py runs and bench.py runs (DLTB_EXT_PATH selects).
#   scripts/ab/ab_attn_v2.sh TAG [TAG...]
set -e
mkdir -p gpurun_out
TAGS=("$@")
SO0=$(ls build/${TAGS[0]}/_C*.so)
DLTB_EXT_PATH=$SO0 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -x -q -k "attn or attention" --timeout 120 --timeout-method thread > gpurun_out/attn_${TAGS[0]}_tests.log 2>&1
tail -3 gpurun_out/attn_${TAGS[0]}_tests.log
for r in 1 2; do
  echo "base:"; timeout -k 10 120 python scripts/bench_attn.py --iters 50 2>&1 | grep -v amdgpu
  for t in "${TAGS[@]}"; do
    echo "$t:"; DLTB_EXT_PATH=$(ls build/$t/_C*.so) timeout -k 10 120 python scripts/bench_attn.py --iters 50 2>&1 | grep -v amdgpu
  done
done
for r in 1 2; do
  echo "bench base: $(timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>&1 | tail -n 1 | grep -o '"ms_per_step": [0-9.]*')"
  echo "bench ${TAGS[0]}: $(DLTB_EXT_PATH=$SO0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>&1 | tail -n 1 | grep -o '"ms_per_step": [0-9.]*')"
done
