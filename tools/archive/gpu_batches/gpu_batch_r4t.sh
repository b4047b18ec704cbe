#!/usr/bin/env bash
# Round-4 GPU check of the tree: the GPU test suite, then the 1-GPU flagship bench twice.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gpu_tests_r4.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_r4.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench_$r.log 2>&1 || exit 1
  tail -n 1 gpurun_out/r4_bench_$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' '; echo
done
