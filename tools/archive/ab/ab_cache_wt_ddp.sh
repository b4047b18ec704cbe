#!/usr/bin/env bash
# A/B: cached W^T in the replicated engines when the optimizer runs every micro-step (DDP with the
# reference's semantics: the transposes are refreshed every step).
set -euo pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
P='import dltb.parallel.replicated as R; o = R.ReplicatedEngine._setup
def s(self):
    o(self); self._cache_wt = False
R.ReplicatedEngine._setup = s'
for r in 1 2 3; do
  for dt in bf16 fp16; do
    timeout -k 10 200 python scripts/ab/ab_patch.py "pass" --strategy ddp --dtype $dt --steps 20 --warmup 5 > gpurun_out/abw_on_$dt.log 2>&1
    timeout -k 10 200 python scripts/ab/ab_patch.py "$P" --strategy ddp --dtype $dt --steps 20 --warmup 5 > gpurun_out/abw_off_$dt.log 2>&1
    echo "run $r ddp $dt cache on: $(tail -n 1 gpurun_out/abw_on_$dt.log | grep -o '"ms_per_step": [0-9.]*')  off: $(tail -n 1 gpurun_out/abw_off_$dt.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
