#!/usr/bin/env bash
# In-step hipBLASLt picks for fc1.fwd + fc2.dgrad (from r6k): interleaved bench + same-box kernel traces
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6l; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
b() { timeout -k 10 200 env "$@" python bench.py --steps 20 --warmup 5 > $O/run.log 2>&1 || return 1; grep -o '"ms_per_step": [0-9.]*' $O/run.log | cut -d' ' -f2; }
for i in 1 2 3; do
  echo "ship $i $(b DLTB_X=0)"
  echo "d1 $i $(b DLTB_BLASLT_FILE=configs/blaslt/ab_instep_fc1_fc2d1.csv)"
  echo "d2 $i $(b DLTB_BLASLT_FILE=configs/blaslt/ab_instep_fc1_fc2d2.csv)"
done
bash scripts/rocprof.sh $O/prof_ship > $O/rp1.log 2>&1 || { tail -20 $O/rp1.log; exit 1; }
DLTB_BLASLT_FILE=configs/blaslt/ab_instep_fc1_fc2d1.csv bash scripts/rocprof.sh $O/prof_d1 > $O/rp2.log 2>&1 || { tail -20 $O/rp2.log; exit 1; }
DLTB_BLASLT_FILE=configs/blaslt/ab_instep_fc1_fc2d2.csv bash scripts/rocprof.sh $O/prof_d2 > $O/rp3.log 2>&1 || { tail -20 $O/rp3.log; exit 1; }
for p in ship d1 d2; do echo "== $p"; sed -n 2,12p $O/prof_$p/summary_steady.txt; grep -E "Cijk|Custom" $O/prof_$p/summary_steady.txt | cut -c1-150; done
