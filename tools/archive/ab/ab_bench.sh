#!/usr/bin/env bash
# A/B a list of bench.py variants in one GPU session (one JSON line each, appended to $OUT).
#   ./scripts/ab/ab_bench.sh OUT.jsonl "ENV=1 --flag" "--other-flag" ...
# Each variant runs as its own process under a time limit; the script stops at the first failure.
set -uo pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="$1"; shift
mkdir -p "$(dirname "$OUT")"
for v in "$@"; do
  envs=(); args=()
  for tok in $v; do
    if [[ "$tok" == *=* && "$tok" != --* ]]; then envs+=("$tok"); else args+=("$tok"); fi
  done
  echo "== variant: $v" >&2
  timeout -k 10 300 env "${envs[@]}" python3 "$ROOT/bench.py" "${args[@]}" >"${OUT%.jsonl}.cur" 2>>"${OUT%.jsonl}.err"
  rc=$?
  if [[ $rc -ne 0 ]]; then echo "variant failed rc=$rc: $v" >&2; exit $rc; fi
  line=$(tail -1 "${OUT%.jsonl}.cur")
  python3 - "$v" "$line" >>"$OUT" <<'EOF'
import json, sys
d = json.loads(sys.argv[2]); d["variant"] = sys.argv[1]; print(json.dumps(d))
print(f"{sys.argv[1]!r:50s} {d['value']:10.0f} tok/s {d['ms_per_step']:.3f} ms", file=sys.stderr)
EOF
done
