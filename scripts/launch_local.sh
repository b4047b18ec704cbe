#!/usr/bin/env bash
# Launch one benchmark configuration on this node with torchrun (one process per MI355X).
# Replaces the reference's K8s launcher (scripts/launch_multi.sh): same flags and defaults.
#
#   ./scripts/launch_local.sh --strategy zero2 --world-size 4 [--seq-len 2048] [--tier A] [--steps 100]
#        [--per-device-batch 1] [--grad-accum 4] [--results-dir results/raw] [-- extra harness flags]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
STRATEGY=""; WS=1; SEQ=2048; TIER=A; STEPS=100; BATCH=1; ACCUM=4; RESULTS="$ROOT/results/raw"
PORT="${MASTER_PORT:-$((29500 + RANDOM % 1000))}"
EXTRA=()
while [[ $# -gt 0 ]]; do
  case "$1" in
    --strategy) STRATEGY="$2"; shift 2 ;;
    --world-size) WS="$2"; shift 2 ;;
    --seq-len) SEQ="$2"; shift 2 ;;
    --tier) TIER="$2"; shift 2 ;;
    --steps) STEPS="$2"; shift 2 ;;
    --per-device-batch) BATCH="$2"; shift 2 ;;
    --grad-accum) ACCUM="$2"; shift 2 ;;
    --results-dir) RESULTS="$2"; shift 2 ;;
    --image|--synthetic) [[ "$1" == "--image" ]] && shift 2 || shift ;;   # accepted for CLI parity, unused
    --) shift; EXTRA=("$@"); break ;;
    *) echo "unknown flag $1" >&2; exit 2 ;;
  esac
done
[[ -z "$STRATEGY" ]] && { echo "--strategy is required (ddp|fsdp|zero2|zero3)" >&2; exit 2; }
ARGS=(--strategy "$STRATEGY" --world-size "$WS" --seq-len "$SEQ" --tier "$TIER" --steps "$STEPS"
      --per-device-batch "$BATCH" --grad-accum "$ACCUM" --results-dir "$RESULTS" --synthetic)
case "$STRATEGY" in
  zero2) ARGS+=(--deepspeed-config "$ROOT/configs/deepspeed/zero2.json") ;;
  zero3) ARGS+=(--deepspeed-config "$ROOT/configs/deepspeed/zero3.json") ;;
  fsdp)  ARGS+=(--fsdp-config "$ROOT/configs/fsdp/fsdp_config.yaml") ;;
esac
export HSA_ENABLE_IPC_MODE_LEGACY="${HSA_ENABLE_IPC_MODE_LEGACY:-0}"
if [[ "$WS" -gt 1 ]]; then
  python -m torch.distributed.run --nnodes 1 --nproc-per-node "$WS" --max-restarts 0 \
       --master-addr 127.0.0.1 --master-port "$PORT" \
       "$ROOT/benchmarking/train_harness.py" "${ARGS[@]}" "${EXTRA[@]}"
else
  python -u "$ROOT/benchmarking/train_harness.py" "${ARGS[@]}" --rank 0 "${EXTRA[@]}"
fi
