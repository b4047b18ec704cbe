#!/bin/bash
# Forward ping-pong A/B (DLTB_FWD_PP, KS = 2) against the release build (KS = 3) and plain KS = 2:
# attention numerics on each ping-pong ring depth, then interleaved microbenchmark rounds at the
# TinyGPT-A shape.  usage: ab_attn_pp.sh "rel ks2 pp pp4 ..." "pp pp4"  (variants, numerics variants)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
VARS=${1:-"rel ks2 pp"}; NUM=${2:-"pp"}
for v in $NUM; do
  DLTB_EXT_PATH=$(ls build/$v/_C*.so) timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q \
    -k "attn or attention" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pp_tests_$v.log 2>&1 \
    || { tail -30 gpurun_out/pp_tests_$v.log; exit 1; }
  echo "$v numerics: $(tail -1 gpurun_out/pp_tests_$v.log)"
done
for r in 1 2 3; do
  for v in $VARS; do
    if [ $v = rel ]; then E=""; else E=$(ls build/$v/_C*.so); fi
    DLTB_EXT_PATH=$E timeout -k 10 120 python scripts/bench_attn.py --iters 50 --shapes tinygpt_a,tinygpt_a_p0 \
      > gpurun_out/pp_${v}_$r.log 2>&1 || { tail -20 gpurun_out/pp_${v}_$r.log; exit 1; }
    echo "$v r$r: $(grep -E ' fwd ' gpurun_out/pp_${v}_$r.log | tr -s ' ' | tr '\n' ' ')"
  done
done
