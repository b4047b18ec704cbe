set -o pipefail
SO=$(ls build/oldmap/_C*.so)
for r in 1 2; do
  for v in new old; do
    for gs in 2 4; do
      if [ $v = old ]; then E=$SO; else E=""; fi
      DLTB_EXT_PATH=$E DLTB_DKDV_GSPLIT=$gs timeout -k 5 120 python scripts/bench_attn.py --shapes m7b --iters 20 > gpurun_out/abd_${v}_${gs}_$r.log 2>&1 || exit 1
      echo "$v gsplit$gs r$r: $(grep -E 'dkdv|total' gpurun_out/abd_${v}_${gs}_$r.log | tr -s ' ' | tr '\n' ' ')"
    done
  done
done
