#!/bin/bash
# Same-box A/B of the headline: the round-3 build (ab_r3/, bench.py + package + libsrnn.so of
# commit 81bd697) against this tree, alternated, driver form (K = 20, W = 5).
#   bash scripts/gpu_ab.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ab}
for i in 1 2 3; do
  (cd ab_r3 && timeout -k 10 300 python bench.py --steps 20 --warmup 5) > gpurun_out/ab_r3_${i}_$TAG.log 2>&1 || exit 1
  echo "r3 $i: $(tail -1 gpurun_out/ab_r3_${i}_$TAG.log | cut -c150-200)"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_r4_${i}_$TAG.log 2>&1 || exit 1
  echo "r4 $i: $(tail -1 gpurun_out/ab_r4_${i}_$TAG.log | cut -c150-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abprof_r3_$TAG -o a --output-format csv -- python3 ab_r3/bench.py \
  --steps 20 --warmup 5 > gpurun_out/abprof_r3_$TAG.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abprof_r4_$TAG -o a --output-format csv -- python3 bench.py \
  --steps 20 --warmup 5 > gpurun_out/abprof_r4_$TAG.log 2>&1 || exit 1
echo "prof ok"
