#!/bin/bash
# Round 4 batch H: split-K pair-fixup NT GEMM -- numerics, then per-product timing vs hipBLASLt for the
# fixup's coherence variants (DLTB_NT_FIXMODE 0 agent-coherent stores/loads, 1 agent fences, 2 no pairing).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "gemm_nt_pair_fixup or gemm_nt_splitk" -p no:cacheprovider > gpurun_out/r4h_tests.log 2>&1 || { tail -30 gpurun_out/r4h_tests.log; exit 1; }
tail -3 gpurun_out/r4h_tests.log
for m in 0 1 2; do
  DLTB_NT_FIXMODE=$m timeout -k 10 300 python -u scripts/bench_gemm_nt.py --fixup > gpurun_out/r4h_gemm_m$m.txt 2>&1 || { tail -30 gpurun_out/r4h_gemm_m$m.txt; exit 1; }
  echo "== fixmode $m"; cat gpurun_out/r4h_gemm_m$m.txt
done
