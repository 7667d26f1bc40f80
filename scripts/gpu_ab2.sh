#!/bin/bash
# Same-box A/B of the headline: ab_base/ (bench.py + package + the previous libsrnn.so) against
# this tree, alternated, driver form (K = 20, W = 5), then a kernel trace of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-abx}
for i in 1 2 3; do
  for V in base new; do
    D=.; [ $V = base ] && D=ab_base
    (cd $D && timeout -k 10 300 python bench.py --steps 20 --warmup 5) > gpurun_out/abx_${V}_${i}_$TAG.log 2>&1 || exit 1
    echo "$V $i: $(tail -1 gpurun_out/abx_${V}_${i}_$TAG.log | cut -c150-200)"
  done
done
