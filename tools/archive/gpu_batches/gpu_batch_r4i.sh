#!/bin/bash
# Round 4 batch I: split-K planes wired into the step (DLTB_SPLITK_PLANES) -- numerics, then an in-step A/B
# of the 1-GPU bench (interleaved), plus the attention forward at KS = 4.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "planes or pair_fixup or splitk or norm" -p no:cacheprovider > gpurun_out/r4i_tests.log 2>&1 \
  || { tail -30 gpurun_out/r4i_tests.log; exit 1; }
tail -1 gpurun_out/r4i_tests.log
for r in 1 2 3; do
  for v in 0 1; do
    DLTB_SPLITK_PLANES=$v timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/r4i_b${v}_$r.log 2>&1 \
      || { tail -20 gpurun_out/r4i_b${v}_$r.log; exit 1; }
    echo "planes=$v r$r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4i_b${v}_$r.log)"
  done
done
for r in 1 2; do
  for v in rel ks4; do
    if [ $v = rel ]; then E=""; else E=$(ls build/$v/_C*.so); fi
    DLTB_EXT_PATH=$E timeout -k 10 120 python scripts/bench_attn.py --iters 50 --shapes tinygpt_a \
      > gpurun_out/r4i_attn_${v}_$r.log 2>&1 || { tail -20 gpurun_out/r4i_attn_${v}_$r.log; exit 1; }
    echo "$v r$r: $(grep -E ' fwd ' gpurun_out/r4i_attn_${v}_$r.log | tr -s ' ')"
  done
done
