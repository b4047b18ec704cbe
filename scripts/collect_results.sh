#!/usr/bin/env bash
# Extract the BENCHMARK_RESULT_JSON block of a run log into <outdir>/<job>_results/result.json
# (the layout parse_metrics globs), plus the harness' extended sidecar when present.
# Replaces the reference's kubectl-logs collector (scripts/collect_results.sh).
#
#   ./scripts/collect_results.sh <log-file> <out-dir> [job-name] [raw-results-dir]
set -euo pipefail
LOG="$1"; OUT="$2"; JOB="${3:-$(basename "$LOG" .log)}"; RAW="${4:-}"
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$OUT/${JOB}_results"
if python3 - "$LOG" "$OUT/${JOB}_results/result.json" <<'PY'
import json, os, sys
sys.path.insert(0, os.environ.get("DLTB_ROOT", "."))
text = open(sys.argv[1], errors="replace").read()
a, b = "BENCHMARK_RESULT_JSON_START", "BENCHMARK_RESULT_JSON_END"
if a not in text:
    sys.exit(1)
rec = json.loads(text.split(a, 1)[1].split(b, 1)[0])
with open(sys.argv[2], "w") as f:
    json.dump(rec, f, indent=2)
PY
then
  echo "collected $OUT/${JOB}_results/result.json"
  if [[ -n "$RAW" ]]; then
    s=$(python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print(f\"result_{r['strategy']}_ws{r['world_size']}_seq{r['seq_len']}_tier{r['tier']}.extended.json\")" "$OUT/${JOB}_results/result.json")
    [[ -f "$RAW/$s" ]] && cp "$RAW/$s" "$OUT/${JOB}_results/result.extended.json"
  fi
else
  echo "no JSON result in $LOG (run failed?)" >&2
  rmdir "$OUT/${JOB}_results" 2>/dev/null || true
  exit 1
fi
