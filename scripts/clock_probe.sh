#!/usr/bin/env bash
# GPU clock / power while the flagship step runs (read-only rocm-smi samples beside bench.py)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/clk
export HSA_ENABLE_IPC_MODE_LEGACY=0
(timeout -k 10 120 python bench.py --steps 6000 --warmup 5 > gpurun_out/clk/bench.log 2>&1) &
BP=$!
sleep 18
for i in 1 2 3 4 5 6; do
  timeout -k 5 20 rocm-smi --showclocks --showpower --showtemp >> gpurun_out/clk/smi.txt 2>&1
  sleep 1
done
wait $BP
rc=$?
timeout -k 5 20 rocm-smi --showclocks --showpower >> gpurun_out/clk/smi_idle.txt 2>&1
tail -1 gpurun_out/clk/bench.log
exit $rc
