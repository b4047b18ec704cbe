#!/usr/bin/env bash
# Round-4 batch G: multi-rank GPU tests (host-staged world 2, eager + lazy), emulated phases and the predicted rows
# of the sharded engines after their tail deferral.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py tests/test_emulate_gpu.py tests/test_graphs_gpu.py -x -q \
    --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/mr_gpu_r4.log 2>&1 || { tail -30 gpurun_out/mr_gpu_r4.log; exit 1; }
tail -2 gpurun_out/mr_gpu_r4.log
for S in zero3 fsdp; do echo "== $S"; STRAT=$S N=8 bash scripts/emu_phases.sh || exit 1; done
STRATS="zero3 fsdp fsdp_root fsdp_bf16" bash scripts/gpu_batch_r4b.sh
