#!/usr/bin/env bash
# DDP early per-bucket AdamW (side stream under the backward): tests, emulated N = 8 A/B and phases
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6g
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_emulate_gpu.py tests/test_multirank_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6g/tests.log 2>&1 || { tail -30 gpurun_out/r6g/tests.log; exit 1; }
tail -1 gpurun_out/r6g/tests.log
for i in 1 2; do
  for v in 0 1; do
    DLTB_DDP_EARLY_OPT=$v timeout -k 10 200 python bench.py --strategy ddp --dtype bf16 --steps 20 --warmup 8 --emulate 8 > gpurun_out/r6g/ddp_e${v}_$i.log 2>&1 || exit 1
    echo "early=$v $i $(tail -n 1 gpurun_out/r6g/ddp_e${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), d.get('comm_wait_ms'))")"
  done
done
STRAT=ddp BASE="--dtype bf16" bash scripts/emu_phases.sh > gpurun_out/r6g/phases.txt 2>&1; cat gpurun_out/r6g/phases.txt
