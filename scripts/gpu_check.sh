#!/usr/bin/env bash
# One GPU-box pass: kernel + model tests, smoke, 1-GPU benches of every strategy, rocprofv3 stats.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out"
mkdir -p "$OUT"
cd "$R"
STEPS="${STEPS:-20}"
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -ra > "$OUT/pytest_gpu.log" 2>&1 \
  && echo "pytest ok" \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  && echo "smoke ok" \
  && for s in ${STRATS:-zero2 ddp fsdp zero3}; do
       timeout -k 10 300 python bench.py --strategy "$s" --steps "$STEPS" --warmup 8 > "$OUT/bench_$s.log" 2>&1 || exit 1
       tail -1 "$OUT/bench_$s.log"
     done \
  && if [ -n "${PROFILE:-}" ]; then
       cd /tmp && export TMPDIR=/tmp && \
       timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
         python3 "$R/bench.py" --strategy zero2 --steps 8 --warmup 4 > "$OUT/prof.log" 2>&1 && echo "profile ok"
     fi
