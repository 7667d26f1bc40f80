#!/bin/bash
# Same-box A/B/C of the headline: round-3 build (ab_r3/), this tree, and this tree with the
# step-by-step permutation decode (ab_v/), alternated, driver form (K = 20, W = 5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ab3}
for i in 1 2 3; do
  for V in r3 r4 v; do
    D=.; [ $V = r3 ] && D=ab_r3; [ $V = v ] && D=ab_v
    (cd $D && timeout -k 10 300 python bench.py --steps 20 --warmup 5) > gpurun_out/ab3_${V}_${i}_$TAG.log 2>&1 || exit 1
    echo "$V $i: $(tail -1 gpurun_out/ab3_${V}_${i}_$TAG.log | cut -c150-200)"
  done
done
