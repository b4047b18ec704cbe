#!/usr/bin/env bash
# Render and submit a Kubernetes run.
#   scripts/launch_multi.sh --strategy zero2 --gpus 8 [--nnodes 1] [--seq-len 2048] [--tier A]
#                           [--steps 100] [--per-device-batch 1] [--grad-accum 4] --image IMG
# --nnodes 1 (default): one pod with all GPUs of a node (k8s/job-node.template.yaml).
# --nnodes > 1: master + Indexed workers Jobs, one pod per node (job-{master,workers}.template.yaml).
set -euo pipefail
STRATEGY=ddp GPUS=8 NNODES=1 SEQ_LEN=2048 TIER=A STEPS=100 WARMUP_STEPS=8 PER_DEVICE_BATCH=1
GRAD_ACCUM=4 IMAGE="${IMAGE:-dltb-mi355x:latest}" GPU_PRODUCT="${GPU_PRODUCT:-AMD_Instinct_MI355X}"
while [ $# -gt 0 ]; do
  case "$1" in
    --strategy) STRATEGY="$2"; shift 2 ;;
    --gpus) GPUS="$2"; shift 2 ;;
    --nnodes) NNODES="$2"; shift 2 ;;
    --seq-len) SEQ_LEN="$2"; shift 2 ;;
    --tier) TIER="$2"; shift 2 ;;
    --steps) STEPS="$2"; shift 2 ;;
    --warmup-steps) WARMUP_STEPS="$2"; shift 2 ;;
    --per-device-batch) PER_DEVICE_BATCH="$2"; shift 2 ;;
    --grad-accum) GRAD_ACCUM="$2"; shift 2 ;;
    --image) IMAGE="$2"; shift 2 ;;
    --synthetic) shift ;;
    *) echo "unknown flag $1" >&2; exit 2 ;;
  esac
done
HERE="$(cd "$(dirname "$0")/.." && pwd)"
JOB_NAME="bench-${STRATEGY}-n${NNODES}x${GPUS}-seq${SEQ_LEN}"
render() {
  sed -e "s|{{JOB_NAME}}|$JOB_NAME|g" -e "s|{{IMAGE}}|$IMAGE|g" -e "s|{{STRATEGY}}|$STRATEGY|g" \
      -e "s|{{GPUS}}|$GPUS|g" -e "s|{{NNODES}}|$NNODES|g" -e "s|{{WORKERS}}|$((NNODES - 1))|g" \
      -e "s|{{SEQ_LEN}}|$SEQ_LEN|g" -e "s|{{TIER}}|$TIER|g" -e "s|{{STEPS}}|$STEPS|g" \
      -e "s|{{WARMUP_STEPS}}|$WARMUP_STEPS|g" -e "s|{{PER_DEVICE_BATCH}}|$PER_DEVICE_BATCH|g" \
      -e "s|{{GRAD_ACCUM}}|$GRAD_ACCUM|g" -e "s|{{GPU_PRODUCT}}|$GPU_PRODUCT|g" "$1"
}
kubectl apply -f "$HERE/k8s/namespace.yaml" -f "$HERE/k8s/serviceaccount.yaml"
if [ "$NNODES" -eq 1 ]; then
  render "$HERE/k8s/job-node.template.yaml" | kubectl apply -f -
else
  kubectl apply -f "$HERE/k8s/service-master.yaml"
  render "$HERE/k8s/job-master.template.yaml" | kubectl apply -f -
  render "$HERE/k8s/job-workers.template.yaml" | kubectl apply -f -
fi
echo "submitted $JOB_NAME  (kubectl -n bench logs -f job/$JOB_NAME)"
