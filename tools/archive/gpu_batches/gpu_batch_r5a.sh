#!/usr/bin/env bash
# Round-5 regression attribution (VERDICT r4 Next #2): interleaved same-box A/B of the round-3 tree
# (5a91585, git worktree build/r3tree with its own in-tree build) against HEAD, 3 rounds each of
# bench.py --steps 20 --warmup 5; then the reference-format harness zero2 row against bench.py on the
# same box (default log cadence, and with the per-10-step loss readback disabled).
set -o pipefail
cd "$(dirname "$0")/.."
ROOT=$(pwd)
mkdir -p gpurun_out/r5a
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5a/smoke.log 2>&1 \
  || { tail -20 gpurun_out/r5a/smoke.log; exit 1; }
tail -1 gpurun_out/r5a/smoke.log
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r5a/head_$r.log 2>&1 || { tail -5 gpurun_out/r5a/head_$r.log; exit 1; }
  echo "HEAD r$r $(tail -n 1 gpurun_out/r5a/head_$r.log)"
  (cd build/r3tree && timeout -k 10 200 python bench.py --steps 20 --warmup 5) > gpurun_out/r5a/r3_$r.log 2>&1 || { tail -5 gpurun_out/r5a/r3_$r.log; exit 1; }
  echo "R3   r$r $(tail -n 1 gpurun_out/r5a/r3_$r.log)"
done
for arm in default nolog; do
  EX=(); [[ $arm == nolog ]] && EX=(--log-every 100000)
  timeout -k 10 300 python -u benchmarking/train_harness.py --strategy zero2 --world-size 1 --rank 0 --tier A \
    --seq-len 2048 --steps 100 --per-device-batch 1 --grad-accum 4 --results-dir gpurun_out/r5a/harness_$arm \
    --deepspeed-config configs/deepspeed/zero2.json "${EX[@]}" > gpurun_out/r5a/harness_$arm.log 2>&1 \
    || { tail -5 gpurun_out/r5a/harness_$arm.log; exit 1; }
  echo "harness $arm: $(grep -h mean_step_time_sec gpurun_out/r5a/harness_$arm/*.json | head -1)"
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r5a/head_4.log 2>&1 && echo "HEAD r4 $(tail -n 1 gpurun_out/r5a/head_4.log)"
