set -e
mkdir -p gpurun_out
echo "== base"; timeout -k 10 120 python scripts/attn_diag.py gpurun_out/diag_base.pt 2>&1 | grep -v amdgpu
echo "== v2";   DLTB_EXT_PATH=$(ls build/attnv2/_C*.so) timeout -k 10 120 python scripts/attn_diag.py gpurun_out/diag_v2.pt 2>&1 | grep -v amdgpu
echo "== base p0"; timeout -k 10 120 python scripts/attn_diag.py gpurun_out/diag_base0.pt 2 256 4 4 64 0 0.0 2>&1 | grep -v amdgpu
echo "== v2 p0";   DLTB_EXT_PATH=$(ls build/attnv2/_C*.so) timeout -k 10 120 python scripts/attn_diag.py gpurun_out/diag_v20.pt 2 256 4 4 64 0 0.0 2>&1 | grep -v amdgpu
