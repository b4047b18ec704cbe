#!/usr/bin/env bash
# Capability runs on one MI355X (bench.py, ZeRO-2, warm-up 8 so the HIP-graph capture stays out of the timed
# steps): Tier B, Tier A at seq 8192 and 32768.  One line per run into gpurun_out/capability_runs.txt.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/capability_runs.txt
: > "$OUT"
run() {
  local tag="$1"; shift
  timeout -k 10 500 python bench.py --warmup 8 "$@" > "gpurun_out/cap_$tag.log" 2>&1 || { echo "$tag FAILED" >> "$OUT"; return 1; }
  python - "$tag" "gpurun_out/cap_$tag.log" >> "$OUT" <<'PY'
import json, sys
tag, path = sys.argv[1], sys.argv[2]
rec = [json.loads(l) for l in open(path) if l.startswith("{")][-1]
print(f"{tag:10s} {rec['config']['model'][:40]:40s} seq {rec['config']['seq_len']:6d}: {rec['value']:9.0f} tok/s "
      f"{rec['ms_per_step']:8.2f} ms/micro-step {rec['peak_hbm_gb']:6.1f} GB {rec['tflops_per_gpu']:5.0f} TFLOP/s")
PY
  tail -1 "$OUT"
}
run tierB --tier B --steps 12 && run a_8k --seq-len 8192 --steps 12 && run a_32k --seq-len 32768 --steps 6
