set -e
SO=$(ls build/prio/_C*.so)
for r in 1 2 3; do
  echo "base:"; timeout -k 10 120 python scripts/bench_attn.py --iters 50 --shapes tinygpt_a 2>&1 | grep -v amdgpu | head -3
  echo "prio:"; DLTB_EXT_PATH=$SO timeout -k 10 120 python scripts/bench_attn.py --iters 50 --shapes tinygpt_a 2>&1 | grep -v amdgpu | head -3
done
bash scripts/pmc_attn.sh gpurun_out/pmc_attn > gpurun_out/pmc_attn.txt 2>&1
grep -A1 "attn_fwd\|attn_bwd_dq\|attn_bwd_dkdv" gpurun_out/pmc_attn.txt
