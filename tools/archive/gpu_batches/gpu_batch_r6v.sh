#!/usr/bin/env bash
# In-step A/B of the workgroup mapping (wgm) of the two MT256x128x64 rows (fc1.fwd, fc2.dgrad)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6v; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
b() { timeout -k 10 200 env "$@" python bench.py --steps 20 --warmup 5 > $O/run.log 2>&1 || return 1; grep -o '"ms_per_step": [0-9.]*' $O/run.log | cut -d' ' -f2; }
for i in 1 2 3; do
  echo "ship $i $(b DLTB_X=0)"
  for w in 1 2 4 8; do echo "wgm$w $i $(b DLTB_BLASLT_FILE=configs/blaslt/ab/wgm${w}_n4096.csv)"; done
done
