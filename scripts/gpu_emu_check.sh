#!/usr/bin/env bash
# GPU-box check of the emulated-fabric comm mode: its GPU tests, then one emulated N=8 ZeRO-2 bench
# with the host-enqueue check.  Outputs under gpurun_out/.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_emulate_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/emu_tests.log 2>&1
rc=$?; tail -15 gpurun_out/emu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --emulate 8 --host-check --steps 20 --warmup 8 > gpurun_out/emu_z2_8.log 2>&1
rc=$?; tail -c 3000 gpurun_out/emu_z2_8.log; exit $rc
