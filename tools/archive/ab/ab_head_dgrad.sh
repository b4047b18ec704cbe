set -e
timeout -k 10 200 python -u -m pytest tests/test_blaslt_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_hd_$r.log 2>&1
  tail -n 1 gpurun_out/bench_hd_$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"mean_loss": [0-9.]*' | tr '\n' ' '; echo
done
DLTB_BLASLT_FILE=none timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_hd_off.log 2>&1
echo -n "table off: "; tail -n 1 gpurun_out/bench_hd_off.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"mean_loss": [0-9.]*' | tr '\n' ' '; echo
