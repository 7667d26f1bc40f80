#!/bin/bash
# Reference-order scheduler check: GPU tests of the ordered generation (+ pairs), the headline
# with its reference-order side measurement, and a kernel trace of both.
#   bash scripts/gpu_r4c.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4c}
timeout -k 10 400 python -u -m pytest tests/test_ordered_soup.py tests/test_pair_soup_gpu.py -m gpu --maxfail=4 -v \
  --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/pytest_$TAG.log | tail -3
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" gpurun_out/pytest_$TAG.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --reference-order-steps -1 > gpurun_out/bench_$TAG.log 2>&1 || exit 1
tail -1 gpurun_out/bench_$TAG.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o sync --output-format csv -- python3 bench.py \
  --steps 20 --warmup 5 --reference-order-steps 20 > gpurun_out/prof_$TAG.log 2>&1 || exit 1
echo "prof ok"
