#!/usr/bin/env bash
# Host cost of an eager emulated-N Mistral-7B ZeRO-3 step, measured on its unit / collective structure at d 512
# (tier M7B_narrow: 32 layers, GQA 4:1, untied head -> the same per-unit gathers, releases, reduce-scatters and
# ProcessGroupNCCL host costs as M7B, negligible GPU work): --host-check holds the GPU and times the enqueue.
# host / GPU for the real shape = this host time / the M7B predicted step (profiles/emulated_m7b_r4.txt).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/m7bhost
for cfg in zero3.json zero3_mi355x_288gb.json; do
  timeout -k 10 300 python bench.py --strategy zero3 --tier M7B_narrow --seq-len 4096 --steps 12 --warmup 8 \
      --emulate 8 --host-check --deepspeed-config configs/deepspeed/$cfg > gpurun_out/m7bhost/$cfg.log 2>&1 || exit 1
  tail -n 1 gpurun_out/m7bhost/$cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', 'gpu ms', round(d['ms_per_step'],2), 'host ms', round(d['host_enqueue_ms_per_step'],2), d.get('host_check_note'))"
done
