#!/usr/bin/env bash
# A/B: cached W^T in the sharded engines at world 1 (FSDP reference semantics: refresh every step).
set -euo pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
P='import dltb.parallel.sharded as S; o = S.ShardedEngine.__init__
def i(self, *a, **k):
    a[1].extra["cache_weight_t"] = False; o(self, *a, **k)
S.ShardedEngine.__init__ = i'
for r in 1 2 3; do
  for st in fsdp zero3; do
    timeout -k 10 200 python scripts/ab/ab_patch.py "pass" --strategy $st --steps 20 --warmup 5 > gpurun_out/abf_on_$st.log 2>&1
    timeout -k 10 200 python scripts/ab/ab_patch.py "$P" --strategy $st --steps 20 --warmup 5 > gpurun_out/abf_off_$st.log 2>&1
    echo "run $r $st cache on: $(tail -n 1 gpurun_out/abf_on_$st.log | grep -o '"ms_per_step": [0-9.]*')  off: $(tail -n 1 gpurun_out/abf_off_$st.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
