set -e
mkdir -p gpurun_out
P='import dltb.parallel.sharded as S; o = S.ShardedEngine.__init__
def i(self, *a, **k):
    a[1].extra["cache_weight_t"] = False; o(self, *a, **k)
S.ShardedEngine.__init__ = i'
for r in 1 2; do
  for st in zero3 fsdp; do
    timeout -k 10 200 python scripts/ab/ab_patch.py "pass" --strategy $st --steps 20 --warmup 5 > gpurun_out/ab_c_on_${st}_$r.log 2>&1
    timeout -k 10 200 python scripts/ab/ab_patch.py "$P" --strategy $st --steps 20 --warmup 5 > gpurun_out/ab_c_off_${st}_$r.log 2>&1
    echo "$st run $r on: $(tail -n 1 gpurun_out/ab_c_on_${st}_$r.log | grep -o '"ms_per_step": [0-9.]*')  off: $(tail -n 1 gpurun_out/ab_c_off_${st}_$r.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
