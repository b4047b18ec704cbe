#!/usr/bin/env bash
# In-step A/B of the own kernel's group-M tile walk (gm) on the five N = 1024 products
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6y; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
b() { timeout -k 10 200 env "$@" python bench.py --steps 20 --warmup 5 > $O/run.log 2>&1 || return 1; grep -o '"ms_per_step": [0-9.]*' $O/run.log | cut -d' ' -f2; }
for i in 1 2 3; do
  echo "ship $i $(b DLTB_X=0)"
  for g in 1 2 4 8; do echo "gm$g $i $(b DLTB_OWN_GEMM_TABLE=configs/gemm_rs/ab_gm$g.csv)"; done
done
