#!/usr/bin/env bash
# Round-4 closing evidence: smoke(), the steady-state kernel profile of the flagship (bench.py as the driver runs
# it, HIP graphs), and the 1-GPU bench twice.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r4z.log 2>&1 \
  || { tail -20 gpurun_out/smoke_r4z.log; exit 1; }
tail -1 gpurun_out/smoke_r4z.log
bash scripts/rocprof.sh gpurun_out/prof_steady_r4z > gpurun_out/rocprof_r4z.log 2>&1 || { tail -20 gpurun_out/rocprof_r4z.log; exit 1; }
head -34 gpurun_out/prof_steady_r4z/summary_steady.txt
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r4z_bench_$r.log 2>&1 || exit 1
  tail -n 1 gpurun_out/r4z_bench_$r.log
done
