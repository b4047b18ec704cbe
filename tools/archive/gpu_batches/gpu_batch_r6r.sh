#!/usr/bin/env bash
# (1) dGELU epilogue A/B again with the new hipBLASLt table (fc2.dgrad on MT256x128 now);
# (2) in-step hipBLASLt candidates for the tied head's three products
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6r; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
b() { timeout -k 10 200 env "$@" python bench.py --steps 20 --warmup 5 > $O/run.log 2>&1 || return 1; grep -o '"ms_per_step": [0-9.]*' $O/run.log | cut -d' ' -f2; }
for i in 1 2 3; do
  echo "ship $i $(b DLTB_X=0)"
  echo "dgelu62 $i $(b DLTB_OWN_GEMM_TABLE=configs/gemm_rs/ab_dgelu62.csv)"
done
timeout -k 10 400 python scripts/instep_blaslt_candidates.py --products head.fwd,head.dgrad,head.wgrad --top 2 --splitk 0,2,4,6,8 --out-dir $O/tables > $O/cands.log 2>&1 || { tail -30 $O/cands.log; exit 1; }
grep "^\[" $O/cands.log
for i in 1 2; do
  echo "ship $i $(b DLTB_X=0)"
  for t in $O/tables/*_[0-9].csv; do
    r=$(b DLTB_BLASLT_FILE=$t) || exit 1
    echo "$(basename $t .csv) $i $r"
  done
done
