#!/usr/bin/env bash
# Round-4 1-GPU reference-format suite (every strategy row through the harness, DS configs read by
# parallel/ds_config.py) -> gpurun_out/suite_1gpu_r4 (CSV, plots, report).
set -o pipefail
cd "$(dirname "$0")/.."
rm -rf gpurun_out/suite_1gpu_r4
STEPS=40 WS_LIST=1 M7B=0 timeout -k 10 1100 bash scripts/run_all_benchmarks.sh gpurun_out/suite_1gpu_r4 > gpurun_out/suite_1gpu_r4.log 2>&1
rc=$?
tail -25 gpurun_out/suite_1gpu_r4.log
cat gpurun_out/suite_1gpu_r4/summary/metrics.csv 2>/dev/null | cut -d, -f1-12
exit $rc
