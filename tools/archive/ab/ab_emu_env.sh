#!/usr/bin/env bash
# A/B of env toggles on the emulated N-rank step (bench.py --emulate N, default alpha-beta model):
#   VARIANTS="NAME:VAR=V,VAR=V NAME2:..." bash scripts/ab/ab_emu_env.sh      (outputs gpurun_out/ab_emu/)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/ab_emu; mkdir -p $O
N="${N:-8}"; S="${STRAT:-zero2}"
for rep in 1 2; do
for v in $VARIANTS; do
  name="${v%%:*}"; envs="${v#*:}"; envs="${envs//,/ }"
  timeout -k 10 200 env $envs python bench.py --strategy $S --steps 20 --warmup 8 --emulate $N $EXTRA > $O/${name}_$rep.log 2>&1 || exit 1
  tail -n 1 $O/${name}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', $rep, round(d['ms_per_step'],3), 'cwait', round(d.get('comm_wait_ms') or 0,3), {k: round(v,3) for k,v in (d.get('phase_ms') or {}).items()}, 'h/g', d.get('host_over_gpu'))"
done
done
