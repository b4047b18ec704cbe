#!/usr/bin/env bash
# Per-kernel A/B of an extension variant (build/TAG) vs the release build: rocprofv3 kernel stats of
# the same short bench, one run each, and the lines of the kernels matching PATTERN.
#   scripts/ab/ab_kernel_times.sh TAG PATTERN [bench flags...]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
TAG=$1; PAT=$2; shift 2
SO=$(ls "$ROOT"/build/$TAG/_C*.so)
cd /tmp && export TMPDIR=/tmp
for v in base "$TAG"; do
  OUT="$ROOT/gpurun_out/abk_$v"
  if [ "$v" = base ]; then E=""; else E="$SO"; fi
  DLTB_EXT_PATH=$E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$ROOT/bench.py" --steps 12 --warmup 4 "$@" > "$OUT.log" 2>&1
  echo "== $v: $(tail -n 1 "$OUT.log" | grep -o '"ms_per_step": [0-9.]*')"
  python3 - "$OUT/run_kernel_stats.csv" "$PAT" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r["Name"]):
        print(f"   {float(r['AverageNs'])/1e3:8.2f} us x {int(r['Calls']):5d}  {r['Name'][:90]}")
PY
done
