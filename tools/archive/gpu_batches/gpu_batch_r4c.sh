#!/usr/bin/env bash
# Round-4 GPU batch C: Mistral-7B-shape ZeRO-3 at emulated N = 8 with the reference's zero3.json (prefetch now an
# element budget, reuse-distance keep) and the 288 GB config; DDP N = 8 solo-tail A/B (VERDICT r3 Next #8).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/abtail
timeout -k 10 900 python scripts/emulated_scaling.py --out gpurun_out/emulated_m7b_r4.txt --strategies --m7b || exit 1
for r in 1 2; do
  for t in 1 4; do
    DLTB_SOLO_TAIL=$t timeout -k 10 200 python bench.py --strategy ddp --emulate 8 --steps 20 --warmup 8 \
        > gpurun_out/abtail/ddp_tail${t}_$r.log 2>&1 || exit 1
    tail -n 1 gpurun_out/abtail/ddp_tail${t}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tail$t', $r, round(d['ms_per_step'],3))"
  done
done
# VERDICT r3 Weak #3: HIP-graph replay of the emulated N = 8 ZeRO-2 step vs eager (graphs drop the tail deferral and
# the carried token rows: collectives may not stay in flight across graph boundaries)
mkdir -p gpurun_out/abgraph
for r in 1 2; do
  for g in off on; do
    timeout -k 10 200 python bench.py --strategy zero2 --emulate 8 --steps 24 --warmup 8 --graphs $g \
        > gpurun_out/abgraph/g${g}_$r.log 2>&1 || exit 1
    tail -n 1 gpurun_out/abgraph/g${g}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('graphs-$g', $r, round(d['ms_per_step'],3), d.get('hip_graphs'))"
  done
done
