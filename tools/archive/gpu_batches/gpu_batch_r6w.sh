#!/usr/bin/env bash
# fc1 forward with the GELU output in the own GEMM's epilogue (table bias = 3): tests + in-step A/B
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6w; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_rs_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
b() { timeout -k 10 200 env "$@" python bench.py --steps 20 --warmup 5 > $O/run.log 2>&1 || return 1; grep -o '"ms_per_step": [0-9.]*' $O/run.log | cut -d' ' -f2; }
for i in 1 2 3; do
  echo "ship $i $(b DLTB_X=0)"
  echo "gelu62 $i $(b DLTB_OWN_GEMM_TABLE=configs/gemm_rs/ab_gelu62.csv)"
  echo "gelu35 $i $(b DLTB_OWN_GEMM_TABLE=configs/gemm_rs/ab_gelu35.csv)"
done
