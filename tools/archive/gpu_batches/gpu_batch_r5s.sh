#!/usr/bin/env bash
# attention tests (causal D=64 dQ at 3 splits from T=1024); DDP bf16 N=8 bucket-tail A/B in emulation
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5s
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k attention > gpurun_out/r5s/attn_tests.log 2>&1 || { tail -20 gpurun_out/r5s/attn_tests.log; exit 1; }
tail -1 gpurun_out/r5s/attn_tests.log
for i in 1 2; do
  for v in "DLTB_SOLO_TAIL=1" "DLTB_SOLO_TAIL=3" "DLTB_SOLO_TAIL=5" "DLTB_BUCKET_UNIT_MULTIPLE=2"; do
    env $v timeout -k 10 200 python bench.py --strategy ddp --dtype bf16 --steps 20 --warmup 8 --emulate 8 > gpurun_out/r5s/ddp_${v}_$i.log 2>&1 || exit 1
    echo "$v $i $(tail -n 1 gpurun_out/r5s/ddp_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), d.get('comm_wait_ms'))")"
  done
done
