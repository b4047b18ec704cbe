#!/usr/bin/env bash
# Pooled gathered buffers + per-buffer view cache (sharded engines) vs fresh buffers: emulated N=8 FSDP and
# ZeRO-3 TinyGPT-A (bench.py --emulate 8 --host-check), alternating on one box.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for r in ${ROUNDS:-1 2}; do
  for s in ${STRATS:-fsdp zero3}; do
    for pool in 1 0; do
      DLTB_GATHER_POOL=$pool timeout -k 10 300 python bench.py --strategy $s --emulate 8 --steps 12 --warmup 8 --host-check > gpurun_out/abgp_${s}_${pool}_$r.log 2>&1 || exit 1
      echo "$s pool=$pool r$r: $(tail -n 1 gpurun_out/abgp_${s}_${pool}_$r.log | grep -o '"predicted_ms_per_step": [0-9.]*\|"host_over_gpu": [0-9.]*\|"host_enqueue_ms_per_step": [0-9.]*' | tr '\n' ' ')"
    done
  done
done
