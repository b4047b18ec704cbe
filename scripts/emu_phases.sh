#!/usr/bin/env bash
# Phase timers (HIP events, eager) of the world-1 step and of the emulated N-rank step -- default
# alpha-beta fabric, a free one (alpha 0, infinite bandwidth), the free one without a traffic stream
# (nocomm: the stand-in kernels still occupy 32 workgroups each), and null (no collective kernel at
# all: the N-rank code path alone; its numerics are not the N-rank ones).
set -o pipefail
cd "$(dirname "$0")/.."
S="${STRAT:-zero2}"; N="${N:-8}"
O=gpurun_out/emu_phases/$S; mkdir -p $O
one() { local name=$1; shift; timeout -k 10 200 env "$@" python bench.py --strategy $S ${BASE:-} --steps 24 --warmup 8 --graphs off $EXTRA > $O/$name.log 2>&1 || return 1
  tail -n 1 $O/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', round(d['ms_per_step'],3), {k: round(v,3) for k,v in (d.get('phase_ms') or {}).items()})"; }
one w1 DLTB_X=0 && EXTRA="--emulate $N" one e${N} DLTB_X=0 && EXTRA="--emulate $N" one e${N}_fast DLTB_EMU_ALPHA_US=0 DLTB_EMU_BUS_GBPS=1e9 &&
EXTRA="--emulate $N" one e${N}_nocomm DLTB_EMU_ALPHA_US=0 DLTB_EMU_BUS_GBPS=1e9 DLTB_EMU_HBM_PASSES=0 &&
EXTRA="--emulate $N" one e${N}_null DLTB_EMU_NULL=1 DLTB_EMU_HOST_US=0
