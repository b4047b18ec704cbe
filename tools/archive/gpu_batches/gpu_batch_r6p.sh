#!/usr/bin/env bash
# ddp_zero1 (DDP + sharded optimizer) bucket-layout A/B on the emulated N = 8 fabric
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6p; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
b() { timeout -k 10 200 env "$@" python bench.py --strategy ddp --dtype bf16 --ddp-shard-optimizer --emulate 8 --steps 20 --warmup 8 > $O/run.log 2>&1 || return 1; tail -n1 $O/run.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), d.get('comm_wait_ms'))"; }
for i in 1 2; do
  echo "tail1 $i $(b DLTB_SOLO_TAIL=1)"
  echo "tail3 $i $(b DLTB_SOLO_TAIL=3)"
  echo "tail5 $i $(b DLTB_SOLO_TAIL=5)"
  echo "mult2 $i $(b DLTB_BUCKET_UNIT_MULTIPLE=2)"
  echo "mult2t3 $i $(b DLTB_BUCKET_UNIT_MULTIPLE=2 DLTB_SOLO_TAIL=3)"
done
