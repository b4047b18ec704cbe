#!/usr/bin/env bash
# In-step A/B of alternative hipBLASLt solutions (other macro tiles) for qkv.fwd, fc1.fwd, fc2.dgrad
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6k; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python scripts/instep_blaslt_candidates.py --top 3 --out-dir $O/tables > $O/cands.log 2>&1 || { tail -30 $O/cands.log; exit 1; }
grep "^\[" $O/cands.log
b() { timeout -k 10 200 env "$@" python bench.py --steps 20 --warmup 5 > $O/run.log 2>&1 || return 1; grep -o '"ms_per_step": [0-9.]*' $O/run.log | cut -d' ' -f2; }
for i in 1 2; do
  echo "ship $i $(b DLTB_X=0)" || exit 1
  for t in $O/tables/*.csv; do
    r=$(b DLTB_BLASLT_FILE=$t) || exit 1
    echo "$(basename $t .csv) $i $r"
  done
done
echo "ship 3 $(b DLTB_X=0)"
