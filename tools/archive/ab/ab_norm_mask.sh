#!/usr/bin/env bash
# A/B: LN1 + attention-dropout mask in one launch (functional.norm_fwd_mask) vs two launches.
set -euo pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
P='import dltb.ops.functional as F
o = F.norm_fwd
F.norm_fwd_mask = lambda x, r, w, b, eps, rms, p, seed, site, y_out, B, T, Hq, pa, asite: (*o(x, r, w, b, eps, rms, p, seed, site, y_out), F.attn_mask(B, T, Hq, pa, seed, asite, x))'
for r in 1 2 3; do
  timeout -k 10 200 python scripts/ab/ab_patch.py "$P" --steps 20 --warmup 5 > gpurun_out/abnm_sep_$r.log 2>&1
  timeout -k 10 200 python scripts/ab/ab_patch.py "pass" --steps 20 --warmup 5 > gpurun_out/abnm_fused_$r.log 2>&1
  echo "run $r separate: $(tail -n 1 gpurun_out/abnm_sep_$r.log | grep -o '"ms_per_step": [0-9.]*')  fused: $(tail -n 1 gpurun_out/abnm_fused_$r.log | grep -o '"ms_per_step": [0-9.]*\|"mean_loss": [0-9.]*' | tr '\n' ' ')"
done
