#!/bin/bash
# Reference-order (level-scheduled) soups and the precomputed permutation table on one MI355X:
# GPU tests of the soups (ordered, fused, sharded), the 100k bench in both orders, and kernel
# traces of both.  Every GPU step has its own timeout; the script stops at the first failure.
#   bash scripts/gpu_ordered.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ord}
timeout -k 10 600 python -u -m pytest tests/test_ordered_soup.py tests/test_sharded_gpu.py tests/test_sharded_multirank_gpu.py \
  tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_sync_$TAG.log 2>&1 && tail -1 gpurun_out/bench_sync_$TAG.log | cut -c1-300 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --order sequential > gpurun_out/bench_seq_$TAG.log 2>&1 && tail -1 gpurun_out/bench_seq_$TAG.log | cut -c1-300 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o ord --output-format csv -- python3 bench.py --steps 20 --warmup 5 --order sequential > gpurun_out/prof_$TAG.log 2>&1 && echo "prof ord ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o sync --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof2_$TAG.log 2>&1 && echo "prof sync ok"
