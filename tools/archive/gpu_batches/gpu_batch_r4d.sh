#!/usr/bin/env bash
# Round-4 GPU batch D: (1) zero2 N=8 under the round-3 emulator settings (1 HBM pass, no host cost) to separate the
# code changes from the emulator changes; (2) M7B ZeRO-3 N=8 with the reference zero3.json: prefetch as an element
# budget (5e8) vs one unit ahead; (3) the multi-fork graph probe.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/d
pr() { python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', round(d['ms_per_step'],3), round(d.get('comm_wait_ms') or 0,3))"; }
for r in 1 2; do
  DLTB_EMU_HBM_PASSES=1 DLTB_EMU_HOST_US=0 timeout -k 10 200 python bench.py --emulate 8 --steps 24 --warmup 8 > gpurun_out/d/z2_r3emu_$r.log 2>&1 || exit 1
  tail -n 1 gpurun_out/d/z2_r3emu_$r.log | pr "zero2-e8-r3emulator-$r"
done
M7="--strategy zero3 --tier M7B --seq-len 4096 --steps 6 --warmup 6 --emulate 8"
timeout -k 10 400 python bench.py $M7 --deepspeed-config configs/deepspeed/zero3.json > gpurun_out/d/m7b_budget.log 2>&1 || exit 1
tail -n 1 gpurun_out/d/m7b_budget.log | pr "m7b-zero3json-budget5e8"
timeout -k 10 400 python bench.py $M7 --deepspeed-config scripts/ab/zero3_prefetch1.json > gpurun_out/d/m7b_pf1.log 2>&1 || exit 1
tail -n 1 gpurun_out/d/m7b_pf1.log | pr "m7b-zero3json-prefetch1"
timeout -k 10 120 python scripts/probes/graph_branch_probe.py > gpurun_out/d/graph_multi.txt 2>&1 || exit 1
grep "graph-branch" gpurun_out/d/graph_multi.txt
