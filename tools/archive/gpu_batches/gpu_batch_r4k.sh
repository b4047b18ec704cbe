#!/bin/bash
# Round 4 batch K: bench.py's own N-rank plumbing at the driver's largest N on one MI355X -- `--gpus 8` launches 8 ranks
# under torch.distributed.run exactly as the driver does, with DLTB_COMM=host so the ranks share cuda:0 through
# host-staged gloo (the tokens/s of such a run means nothing; the JSON line, timing bracket and max-over-ranks do).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
DLTB_COMM=host timeout -k 10 900 python bench.py --gpus 8 --steps 2 --warmup 2 > gpurun_out/r4k_bench8.log 2>&1; rc=$?
grep -E "^\{|Error|error" gpurun_out/r4k_bench8.log | cut -c1-900 | tail -5
exit $rc
