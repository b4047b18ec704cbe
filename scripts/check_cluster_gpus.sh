#!/usr/bin/env bash
# Kubernetes cluster readiness for MI355X jobs (reference: scripts/check_cluster_gpus.sh, which checks
# an OKE cluster's NVIDIA plugin). Checks, in order:
#   1. kubectl can reach the cluster;
#   2. the AMD GPU device plugin (or the AMD GPU operator) is running;
#   3. nodes advertising `amd.com/gpu`: capacity, allocatable, product label (MI355X expected);
#   4. GPUs already requested by running pods;
#   5. the `bench` namespace, its service account and the image pull secret of k8s/.
# Node-level checks (rocm-smi, xGMI topology, RCCL, the built extension) are in scripts/check_gpus.sh.
set -uo pipefail
NS="${NAMESPACE:-bench}"
SECRET="${PULL_SECRET:-registry-secret}"
RES="amd.com/gpu"
fail=0

echo "== 1. cluster connectivity"
if ! kubectl cluster-info >/dev/null 2>&1; then
  echo "ERROR: kubectl cannot reach a cluster (configure KUBECONFIG)"; exit 1
fi
echo "context: $(kubectl config current-context)"

echo "== 2. AMD GPU device plugin / operator"
plug=$(kubectl get pods -A -l name=amdgpu-dp-ds -o name 2>/dev/null | wc -l)
[[ "$plug" -eq 0 ]] && plug=$(kubectl get pods -A -o name 2>/dev/null | grep -c -E "amdgpu-device-plugin|amd-gpu-operator|device-plugin.*amd" || true)
if [[ "$plug" -eq 0 ]]; then
  echo "ERROR: no AMD GPU device plugin or operator pods found"; fail=1
else
  echo "device plugin / operator pods: $plug"
fi

echo "== 3. GPU nodes"
if command -v jq >/dev/null; then
  kubectl get nodes -o json | jq -r --arg r "$RES" '
    .items[] | select(.status.capacity[$r] != null) |
    [.metadata.name, .status.capacity[$r], .status.allocatable[$r],
     (.metadata.labels["amd.com/gpu.product-name"] // .metadata.labels["node.kubernetes.io/instance-type"] // "unknown")] | @tsv' |
    awk 'BEGIN{printf "%-36s %8s %12s  %s\n","node","capacity","allocatable","product"} {printf "%-36s %8s %12s  %s\n",$1,$2,$3,$4; c+=$2; a+=$3} END{printf "total capacity %d, allocatable %d\n",c,a; if (c==0) exit 3}' || { echo "ERROR: no node advertises $RES"; fail=1; }
else
  kubectl describe nodes | grep -E "^Name:|${RES}" || { echo "ERROR: no node advertises $RES"; fail=1; }
fi

echo "== 4. GPUs requested by running pods"
if command -v jq >/dev/null; then
  kubectl get pods -A -o json | jq -r --arg r "$RES" '
    [.items[] | select(.status.phase=="Running") | .spec.containers[] | (.resources.limits[$r] // "0") | tonumber] | add // 0' |
    xargs -I{} echo "in use: {}"
fi

echo "== 5. namespace, service account, pull secret"
kubectl get ns "$NS" >/dev/null 2>&1 && echo "namespace $NS: ok" || echo "namespace $NS: missing (kubectl apply -f k8s/namespace.yaml)"
kubectl -n "$NS" get sa bench-sa >/dev/null 2>&1 && echo "serviceaccount bench-sa: ok" || echo "serviceaccount bench-sa: missing (k8s/serviceaccount.yaml)"
kubectl -n "$NS" get secret "$SECRET" >/dev/null 2>&1 && echo "secret $SECRET: ok" || echo "secret $SECRET: missing (only needed for private registries)"

if [[ $fail -ne 0 ]]; then echo "CLUSTER NOT READY"; exit 1; fi
echo "CLUSTER READY for MI355X benchmark jobs"
