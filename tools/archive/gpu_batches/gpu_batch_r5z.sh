#!/usr/bin/env bash
# cold weights: XCD-sliced tile walk (own kernel gm = 16) and hipBLASLt workgroup-mapping variants, in-step A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5z gpurun_out/r5z/blt
# hipBLASLt variants: the wide-N per-layer rows (fc1 fwd, fc2 dgrad, qkv fwd) at workgroup mapping W
for w in 4 8 16 32; do
  awk -F, -v W=$w 'BEGIN{OFS=","} NR==1{print;next} ($1=="bf16" && $7==1 && $2==1 && $3==0 && (($4==4096&&$5==2048&&$6==1024) || ($4==3072&&$5==2048&&$6==1024))){$18=W} {print}' \
    configs/blaslt/blaslt_gfx950.csv > gpurun_out/r5z/blt/wgm$w.csv
done
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python scripts/bench_gemm_rs.py --iters 30 --gm 1,4,16 --cfgs 34,62,64 --cold > gpurun_out/r5z/rs_cold.txt 2>&1 || exit 1
run() { local tag=$1; shift; env "$@" timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r5z/bench_${tag}_$i.log 2>&1; }
for i in 1 2; do
  run ship DLTB_X=0 || exit 1
  run g16 DLTB_OWN_GEMM_TABLE=configs/gemm_rs/ab_rsf_g16.csv || exit 1
  run g16all DLTB_OWN_GEMM_TABLE=configs/gemm_rs/ab_rsf_g16all.csv || exit 1
  for w in 4 8 16 32; do run wgm$w DLTB_BLASLT_FILE=gpurun_out/r5z/blt/wgm$w.csv || exit 1; done
done
for f in gpurun_out/r5z/bench_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
