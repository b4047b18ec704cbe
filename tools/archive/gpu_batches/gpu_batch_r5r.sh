#!/usr/bin/env bash
# fenced direct-operand gemm_rsg: correctness, timing; then the DDP pipeline phases / predicted rows
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5r
export HSA_ENABLE_IPC_MODE_LEGACY=0
CFGS=52,53,54,55,56,57,58 REPS=3 timeout -k 10 200 python scripts/debug_gemm_rs.py > gpurun_out/r5r/debug.txt 2>&1 || { cat gpurun_out/r5r/debug.txt; exit 1; }
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 50 --gm 1,4 --cfgs 34,52,53,54,55,56,57,58 > gpurun_out/r5r/rs_warm.txt 2>&1 || exit 1
SO=$(ls build/kscap0/_C*.so)
for i in 1 2; do
  timeout -k 10 120 python scripts/bench_attn.py --shapes causal_d64,causal_d64_short >> gpurun_out/r5r/attn_cap.txt 2>&1 || exit 1
  DLTB_EXT_PATH=$PWD/$SO timeout -k 10 120 python scripts/bench_attn.py --shapes causal_d64,causal_d64_short >> gpurun_out/r5r/attn_nocap.txt 2>&1 || exit 1
done
bash scripts/gpu_batch_r5q.sh
