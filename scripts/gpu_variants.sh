#!/bin/bash
# A/B of env-var variants of the headline bench: one bench.py run per variant.
# usage: gpu_variants.sh TAG "VAR=val VAR2=val" "VAR=val" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
for v in "$@"; do
  env $v timeout -k 10 200 python bench.py --steps 400 --warmup 10 > gpurun_out/var_${TAG}.log 2>&1 || { echo "variant [$v] failed"; tail -5 gpurun_out/var_${TAG}.log; exit 1; }
  echo "[$v] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/var_${TAG}.log)"
done
