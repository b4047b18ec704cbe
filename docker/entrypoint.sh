#!/usr/bin/env bash
# Container entrypoint: environment -> harness command line.
#
# Single node (the MI355X layout): NPROC_PER_NODE GPUs of this pod run one rank each under
# torch.distributed.run (c10d rendezvous on 127.0.0.1, RCCL over xGMI).  Multi-node K8s jobs
# (k8s/job-*.template.yaml) set NNODES / NODE_RANK / MASTER_ADDR and the same script launches
# this node's ranks.  Defaults mirror the reference entrypoint's variables.
set -uo pipefail

STRATEGY="${STRATEGY:-ddp}"
NPROC_PER_NODE="${NPROC_PER_NODE:-${GPUS:-1}}"
NNODES="${NNODES:-1}"
if [ -n "${JOB_COMPLETION_INDEX:-}" ]; then NODE_RANK=$((JOB_COMPLETION_INDEX + 1)); else NODE_RANK="${NODE_RANK:-0}"; fi
if [ "$NODE_RANK" = "0" ] && [ -n "${POD_IP:-}" ]; then MASTER_ADDR="$POD_IP"; fi
MASTER_ADDR="${MASTER_ADDR:-127.0.0.1}"
MASTER_PORT="${MASTER_PORT:-29500}"
SEQ_LEN="${SEQ_LEN:-2048}"
TIER="${TIER:-A}"
STEPS="${STEPS:-50}"
WARMUP_STEPS="${WARMUP_STEPS:-5}"
PER_DEVICE_BATCH="${PER_DEVICE_BATCH:-1}"
GRAD_ACCUM="${GRAD_ACCUM:-1}"
RESULTS_DIR="${RESULTS_DIR:-/results}"
APP="${APP:-/app}"
EXTRA_ARGS="${EXTRA_ARGS:-}"

echo "=== dltb entrypoint $(date) ==="
echo "strategy=$STRATEGY nnodes=$NNODES node_rank=$NODE_RANK nproc_per_node=$NPROC_PER_NODE master=$MASTER_ADDR:$MASTER_PORT"
echo "seq_len=$SEQ_LEN tier=$TIER steps=$STEPS warmup=$WARMUP_STEPS batch=$PER_DEVICE_BATCH accum=$GRAD_ACCUM"
rocm-smi --showproductname 2>/dev/null | grep -E "GPU\[|Card" | head -8 || echo "WARNING: rocm-smi unavailable"

ARGS=(--strategy "$STRATEGY" --seq-len "$SEQ_LEN" --tier "$TIER" --steps "$STEPS"
      --warmup-steps "$WARMUP_STEPS" --per-device-batch "$PER_DEVICE_BATCH" --grad-accum "$GRAD_ACCUM"
      --results-dir "$RESULTS_DIR" --synthetic)
case "$STRATEGY" in
  zero2) ARGS+=(--deepspeed-config "$APP/configs/deepspeed/zero2.json") ;;
  zero3) ARGS+=(--deepspeed-config "$APP/configs/deepspeed/zero3.json") ;;
  fsdp)  ARGS+=(--fsdp-config "$APP/configs/fsdp/fsdp_config.yaml") ;;
esac
# shellcheck disable=SC2206
ARGS+=($EXTRA_ARGS)

WORLD=$((NNODES * NPROC_PER_NODE))
if [ "$WORLD" -gt 1 ]; then
  CMD=(python3 -u -m torch.distributed.run --nnodes "$NNODES" --node-rank "$NODE_RANK"
       --nproc-per-node "$NPROC_PER_NODE" --master-addr "$MASTER_ADDR" --master-port "$MASTER_PORT"
       --max-restarts 0 "$APP/benchmarking/train_harness.py" "${ARGS[@]}")
else
  CMD=(python3 -u "$APP/benchmarking/train_harness.py" --world-size 1 --rank 0 "${ARGS[@]}")
fi
echo "=== launching: ${CMD[*]}"
# a child process (no exec): the shell stays the container's PID 1 and returns the exit code
"${CMD[@]}"
rc=$?
echo "=== training exited with $rc"
exit $rc
