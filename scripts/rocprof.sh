#!/usr/bin/env bash
# Kernel-level profile of the flagship step with rocprofv3 (kernel trace + stats, CSV) and a summary.
#   ./scripts/rocprof.sh [out-dir] [bench.py flags...]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${1:-$ROOT/gpurun_out/prof}"; shift || true
mkdir -p "$OUT"
OUT="$(cd "$OUT" && pwd)"          # absolute: the profiler runs from /tmp
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 "$ROOT/bench.py" --steps 8 --warmup 4 "$@"
python3 "$ROOT/scripts/prof_summary.py" "$OUT" 12 > "$OUT/summary_all.txt"
python3 "$ROOT/scripts/prof_summary.py" "$OUT" --steady | tee "$OUT/summary_steady.txt"
