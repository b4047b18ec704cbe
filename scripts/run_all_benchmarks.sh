#!/usr/bin/env bash
# Full benchmark suite on one 8x MI355X node: every strategy at 1/2/4/8 GPUs (reference:
# scripts/run_all_benchmarks.sh ran {ddp,fsdp,zero2,zero3} x WS{2,4} as K8s jobs).
# Each config: launch (torchrun) -> collect -> failure bookkeeping; then parse -> plot -> report.
# Like the reference it always exits 0; failed configs are listed in results/summary/failures.json.
#
#   ./scripts/run_all_benchmarks.sh [results-dir]
#   env: STEPS, SEQ, TIER, WS_LIST, STRATS, TIMEOUT, HARNESS_EXTRA (extra harness flags),
#        FORCE_NPROC (process slots when no GPU is visible, e.g. the gloo/CPU rehearsal)
set -uo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
RESULTS="${1:-$ROOT/results}"
STEPS="${STEPS:-100}"; SEQ="${SEQ:-2048}"; TIER="${TIER:-A}"; TIMEOUT="${TIMEOUT:-900}"
STRATS="${STRATS:-ddp fsdp zero2 zero3}"
NGPU="${FORCE_NPROC:-$(python3 -c "import torch; print(torch.cuda.device_count())" 2>/dev/null || echo 0)}"
read -r -a HX <<< "${HARNESS_EXTRA:-}"
WS_LIST="${WS_LIST:-1 2 4 8}"
mkdir -p "$RESULTS/raw" "$RESULTS/summary"
FAILED=(); DONE=0
echo "=================================================================="
echo "  MI355X Distributed Training Benchmark Suite ($NGPU GPUs visible)"
echo "=================================================================="
for s in $STRATS; do
  for ws in $WS_LIST; do
    if [[ "$ws" -gt "$NGPU" ]]; then echo "skip $s ws=$ws (only $NGPU GPUs)"; continue; fi
    job="bench-master-${s}-ws${ws}-seq${SEQ}"
    echo "---- $job"
    if timeout -k 30 "$TIMEOUT" "$ROOT/scripts/launch_local.sh" --strategy "$s" --world-size "$ws" --seq-len "$SEQ" \
         --tier "$TIER" --steps "$STEPS" --per-device-batch 1 --grad-accum 4 --results-dir "$RESULTS/raw" -- "${HX[@]}" \
         > "$RESULTS/$job.log" 2>&1 \
       && "$ROOT/scripts/collect_results.sh" "$RESULTS/$job.log" "$RESULTS" "$job" "$RESULTS/raw"; then
      DONE=$((DONE + 1)); echo "     ok"
    else
      FAILED+=("$job"); echo "     FAILED (see $RESULTS/$job.log)"; tail -20 "$RESULTS/$job.log" || true
    fi
  done
done
python3 - "$RESULTS/summary/failures.json" "${FAILED[@]}" <<'PY'
import json, sys
json.dump({"failed": sys.argv[2:]}, open(sys.argv[1], "w"), indent=2)
PY
python3 "$ROOT/scripts/parse_metrics.py" --results-dir "$RESULTS" --out "$RESULTS/summary" \
  && python3 "$ROOT/scripts/plot.py" --results "$RESULTS/summary/metrics.csv" --out "$RESULTS/summary/plots" \
  && python3 "$ROOT/scripts/make_report.py" --csv "$RESULTS/summary/metrics.csv" --out "$RESULTS/summary"
echo "completed: $DONE, failed: ${#FAILED[@]}"
exit 0
