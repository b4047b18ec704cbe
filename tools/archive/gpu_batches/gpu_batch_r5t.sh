#!/usr/bin/env bash
# 1-GPU multi-sequence-length suite: the reference's strategies at seq 2048/4096/8192 (+ Tier B
# long-sequence rows), CSV + report + all plots
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -rf gpurun_out/suite_multiseq
BENCHMARKS_FILE=configs/suite/multiseq_1gpu.txt WS_LIST=1 M7B=0 TIMEOUT=300 timeout -k 10 1150 \
  bash scripts/run_all_benchmarks.sh gpurun_out/suite_multiseq > gpurun_out/suite_multiseq.log 2>&1
rc=$?
tail -25 gpurun_out/suite_multiseq.log
ls gpurun_out/suite_multiseq/summary gpurun_out/suite_multiseq/summary/plots 2>/dev/null
exit $rc
