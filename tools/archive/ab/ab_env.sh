#!/usr/bin/env bash
# Per-kernel + bench A/B of an environment switch: rocprofv3 kernel stats of a short bench with
# VAR=A and VAR=B (kernels matching PATTERN), then ROUNDS interleaved bench.py runs of each.
#   scripts/ab/ab_env.sh VAR A B PATTERN ROUNDS [bench flags...]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
VAR=$1; A=$2; B=$3; PAT=$4; ROUNDS=$5; shift 5
cd /tmp && export TMPDIR=/tmp
for v in "$A" "$B"; do
  OUT="$ROOT/gpurun_out/abenv_${VAR}_$v"
  env "$VAR=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$ROOT/bench.py" --steps 12 --warmup 4 "$@" > "$OUT.log" 2>&1
  echo "== $VAR=$v: $(tail -n 1 "$OUT.log" | grep -o '"ms_per_step": [0-9.]*')"
  python3 - "$OUT/run_kernel_stats.csv" "$PAT" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r["Name"]):
        print(f"   {float(r['AverageNs'])/1e3:8.2f} us x {int(r['Calls']):5d}  {r['Name'][:90]}")
PY
done
for i in $(seq "$ROUNDS"); do
  for v in "$A" "$B"; do
    L="$ROOT/gpurun_out/abenv_bench_${v}_$i.log"
    env "$VAR=$v" timeout -k 10 200 python3 "$ROOT/bench.py" --steps 40 --warmup 8 "$@" > "$L" 2>&1
    echo "bench $VAR=$v round $i: $(tail -n 1 "$L" | grep -o '"ms_per_step": [0-9.]*')"
  done
done
