#!/usr/bin/env bash
# Round-5 checkpoint: full GPU test suite, smoke(), bench twice (own-GEMM table shipped)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5n
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5n/gpu_tests.log 2>&1 \
  || { tail -30 gpurun_out/r5n/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r5n/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5n/smoke.log 2>&1 || { tail -20 gpurun_out/r5n/smoke.log; exit 1; }
tail -1 gpurun_out/r5n/smoke.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r5n/bench_$r.log 2>&1 || exit 1
  tail -n 1 gpurun_out/r5n/bench_$r.log
done
