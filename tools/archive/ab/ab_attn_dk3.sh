#!/bin/bash
# dK/dV with 3 query splits per workgroup at D = 64 (12 waves, 168 VGPRs, 80 B scratch) vs the release 2 splits:
# attention numerics on the dk3 build, then interleaved microbenchmark rounds at the TinyGPT-A shape.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
E=$(ls build/dk3/_C*.so)
DLTB_EXT_PATH=$E timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attn or attention" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dk3_tests.log 2>&1 || { tail -30 gpurun_out/dk3_tests.log; exit 1; }
echo "dk3 numerics: $(tail -1 gpurun_out/dk3_tests.log)"
for r in 1 2 3; do
  for v in rel dk3; do
    if [ $v = rel ]; then X=""; else X=$E; fi
    DLTB_EXT_PATH=$X timeout -k 10 120 python scripts/bench_attn.py --iters 50 --shapes tinygpt_a \
      > gpurun_out/dk3_${v}_$r.log 2>&1 || { tail -20 gpurun_out/dk3_${v}_$r.log; exit 1; }
    echo "$v r$r: $(grep -E ' dkdv ' gpurun_out/dk3_${v}_$r.log | tr -s ' ')"
  done
done
