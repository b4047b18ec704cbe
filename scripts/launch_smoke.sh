#!/usr/bin/env bash
# Submit the 1-GPU smoke job with IMAGE substituted.  IMAGE=... scripts/launch_smoke.sh
set -euo pipefail
IMAGE="${IMAGE:-dltb-mi355x:latest}"
HERE="$(cd "$(dirname "$0")/.." && pwd)"
kubectl apply -f "$HERE/k8s/namespace.yaml" -f "$HERE/k8s/serviceaccount.yaml"
sed "s|__IMAGE__|$IMAGE|g" "$HERE/k8s/job-smoke-1gpu.yaml" | kubectl apply -f -
echo "kubectl -n bench logs -f job/dltb-smoke-1gpu"
