#!/usr/bin/env bash
# colpart row-batching A/B (profiles/colpart_batch_ab_r3.txt): needs build/cp1 = python csrc/build.py --tag cp1 -D DLTB_COLPART_BATCH=1
# against a release build with the batched loop (the experiment; the shipped loop has no such macro any more)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "colpart or gelu or norm or dropout or colreduce" > gpurun_out/t_cp.log 2>&1 || exit 1
bash scripts/ab/ab_ext.sh cp1 3 > gpurun_out/ab_cp.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cp4 -o run -- python bench.py --steps 8 --warmup 5 > gpurun_out/prof_cp4.log 2>&1 || exit 1
DLTB_EXT_PATH=$(ls build/cp1/_C*.so) timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cp1 -o run -- python bench.py --steps 8 --warmup 5 > gpurun_out/prof_cp1.log 2>&1
