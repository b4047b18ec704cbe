#!/usr/bin/env bash
# Build the MI355X image (docker/Dockerfile).  IMAGE=<registry>/<repo>:<tag> scripts/build.sh
set -euo pipefail
IMAGE="${IMAGE:-dltb-mi355x:latest}"
cd "$(dirname "$0")/.."
docker build -f docker/Dockerfile -t "$IMAGE" ${BASE:+--build-arg BASE="$BASE"} .
echo "built $IMAGE"
