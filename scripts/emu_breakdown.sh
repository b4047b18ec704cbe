#!/usr/bin/env bash
# Where does the emulated N-rank step lose time?  ZeRO-2 TinyGPT-A, 1 GPU: the real world-1 step,
# then emulate:8 with (a) an infinitely fast fabric (the N-rank code path alone), (b) the default
# alpha-beta model with 1 channel (duration without CU occupancy), (c) the default model with
# 32 channels.  Outputs under gpurun_out/emu_breakdown/.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/emu_breakdown; mkdir -p $O
S="${STRAT:-zero2}"
run() { local name=$1; shift; timeout -k 10 200 env "$@" python bench.py --strategy $S --steps 20 --warmup 8 $EXTRA > $O/$name.log 2>&1 || return 1
  tail -n 1 $O/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', round(d['ms_per_step'],3), 'cwait', d.get('comm_wait_ms'), 'phases', {k: round(v,3) for k,v in (d.get('phase_ms') or {}).items()}, 'host/gpu', d.get('host_over_gpu'))"; }
run w1 DLTB_X=0 && \
EXTRA="--emulate 8 --host-check" run e8_fast DLTB_EMU_ALPHA_US=0 DLTB_EMU_BUS_GBPS=1e9 && \
EXTRA="--emulate 8" run e8_ch1 DLTB_EMU_CHANNELS=1 && \
EXTRA="--emulate 8" run e8_ch32 DLTB_EMU_CHANNELS=32 && \
EXTRA="--emulate 8 --graphs on" run e8_graphs DLTB_GRAPHS=1
