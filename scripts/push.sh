#!/usr/bin/env bash
# Push the image built by scripts/build.sh.  IMAGE=<registry>/<repo>:<tag> scripts/push.sh
set -euo pipefail
IMAGE="${IMAGE:-dltb-mi355x:latest}"
docker push "$IMAGE"
