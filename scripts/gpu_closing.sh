#!/bin/bash
# A/B of the headline against ab_base/ (same box), then the round-4 closing check.
#   bash scripts/gpu_closing.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-close}
bash scripts/gpu_ab2.sh $TAG || exit $?
bash scripts/gpu_final4.sh $TAG
