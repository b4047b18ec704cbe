#!/usr/bin/env bash
# DDP early per-bucket AdamW with a capped grid (trickle beside the backward): tests + emulated N = 8 A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6h
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k adamw tests/test_emulate_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6h/tests.log 2>&1 || { tail -30 gpurun_out/r6h/tests.log; exit 1; }
tail -1 gpurun_out/r6h/tests.log
for i in 1 2; do
  for v in off 0 32 64 128; do
    if [ $v = off ]; then E=0; G=0; else E=1; G=$v; fi
    DLTB_DDP_EARLY_OPT=$E DLTB_DDP_EARLY_GRID=$G timeout -k 10 200 python bench.py --strategy ddp --dtype bf16 --steps 20 --warmup 8 --emulate 8 > gpurun_out/r6h/ddp_$v_$i.log 2>&1 || exit 1
    echo "early=$v $i $(tail -n 1 gpurun_out/r6h/ddp_$v_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3))")"
  done
done
