#!/usr/bin/env bash
# Window dW (K = 8192, 16-batch) hipBLASLt rows: the recorded keys, then an in-step wgm A/B
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6aa; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python - > $O/keys.log 2>&1 <<'PY' || { tail -20 $O/keys.log; exit 1; }
import argparse, sys, os
sys.path.insert(0, "scripts"); sys.path.insert(0, ".")
os.environ["DLTB_BLASLT_FILE"] = "none"
from tune_blaslt import record_problems
probs, keep = record_problems(argparse.Namespace(tier="A", seq_len=2048, strategy="zero2", dtype="bf16", grad_accum=4, emulate=0))
for k in probs:
    if k[5] == 8192 or k[6] > 1:
        print("KEY", ",".join(str(x) for x in k))
PY
grep KEY $O/keys.log
b() { timeout -k 10 200 env "$@" python bench.py --steps 20 --warmup 5 > $O/run.log 2>&1 || return 1; grep -o '"ms_per_step": [0-9.]*' $O/run.log | cut -d' ' -f2; }
for i in 1 2 3; do
  echo "ship $i $(b DLTB_X=0)"
  for w in 0 8 16; do echo "dw_wgm$w $i $(b DLTB_BLASLT_FILE=configs/blaslt/ab/dw_window_wgm$w.csv)"; done
done
