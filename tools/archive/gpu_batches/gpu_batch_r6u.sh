#!/usr/bin/env bash
# Reference-format 1-GPU suite on the final round-5 tree (the README's suite table)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/suite1_r5; rm -rf $O; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=40 WS_LIST=1 M7B=0 COLLECTIVES=0 TIMEOUT=300 timeout -k 10 1000 bash scripts/run_all_benchmarks.sh $O > $O/suite.log 2>&1 || { tail -20 $O/suite.log; exit 1; }
cat $O/summary/failures.json
cut -d, -f1-8 $O/summary/metrics.csv
