#!/usr/bin/env bash
# Shared column-sum reducer for ZeRO-3 / FSDP at world 1: tests + zero3 / fsdp bench A/B
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6z; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_graphs_gpu.py tests/test_mistral_gpu.py tests/test_fp16_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
b() { timeout -k 10 200 env "$@" > $O/run.log 2>&1 || return 1; grep -o '"ms_per_step": [0-9.]*' $O/run.log | cut -d' ' -f2; }
for i in 1 2; do
  for s in zero3 fsdp; do
    echo "$s red0 $i $(b DLTB_SHARED_RED=0 python bench.py --strategy $s --steps 20 --warmup 8)"
    echo "$s red1 $i $(b DLTB_SHARED_RED=1 python bench.py --strategy $s --steps 20 --warmup 8)"
  done
done
