#!/usr/bin/env bash
# Re-tune the hipBLASLt GEMM selections (PyTorch TunableOp) for the TinyGPT shapes on one GPU and
# write configs/tunableop/tunableop_results_gfx950.csv.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
DLTB_TUNABLEOP_FILE="${1:-$ROOT/configs/tunableop/tunableop_results_gfx950.csv}" \
  python3 "$ROOT/bench.py" --tunableop tune --graphs off --steps 8 --warmup 4
