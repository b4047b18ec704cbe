set -e
mkdir -p gpurun_out
SO=$(ls build/mpad/_C*.so)
DLTB_EXT_PATH=$SO timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -x -q -k "attn or attention" --timeout 120 --timeout-method thread > gpurun_out/mpad_tests.log 2>&1
for r in 1 2 3; do
  echo "base:"; timeout -k 10 120 python scripts/bench_attn.py --iters 50 2>&1 | grep -v amdgpu
  echo "mpad:"; DLTB_EXT_PATH=$SO timeout -k 10 120 python scripts/bench_attn.py --iters 50 2>&1 | grep -v amdgpu
done
cd /tmp && export TMPDIR=/tmp
DLTB_EXT_PATH=$GRAFT_REPO_ROOT/$SO timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_mpad -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_attn.py --iters 5 --shapes tinygpt_a > $GRAFT_REPO_ROOT/gpurun_out/pmc_mpad.log 2>&1
python3 $GRAFT_REPO_ROOT/scripts/pmc_table.py $GRAFT_REPO_ROOT/gpurun_out/pmc_mpad --match attn
