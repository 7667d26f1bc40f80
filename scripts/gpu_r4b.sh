#!/bin/bash
# Round-4 check of the pending-record level scheduler and the permutation-table policy:
#   1. GPU tests of the reference-order generation, lane pairs, sharded soups
#   2. the 1-GPU headline (driver form, K = 20) with its reference-order side measurement
#   3. kernel trace of the headline + reference-order run
#   4. table on / off x lanes per particle over population sizes (both orders)
#   5. strong-scaling model of one rank at N = 8 with and without the table
# Every GPU step has its own timeout; a fault / abort / timeout ends the script.
#   bash scripts/gpu_r4b.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4b}
timeout -k 10 600 python -u -m pytest tests/test_ordered_soup.py tests/test_pair_soup_gpu.py tests/test_sharded_gpu.py \
  tests/test_bench_contract_gpu.py -m gpu --maxfail=6 -v --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/pytest_$TAG.log | tail -3
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" gpurun_out/pytest_$TAG.log | head -20; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --reference-order-steps -1 > gpurun_out/bench_$TAG.log 2>&1 || exit 1
tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o sync --output-format csv -- python3 bench.py \
  --steps 20 --warmup 5 --reference-order-steps 20 > gpurun_out/prof_$TAG.log 2>&1 || exit 1
echo "prof ok"
timeout -k 10 420 python -u bench/pair_sweep.py --sizes 12500,25000,50000,100000 --tables 0,1 \
  > gpurun_out/pairs_$TAG.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/pairs_$TAG.log | cut -c1-130
for PT in 0 1; do
  SRNN_PERM_TABLE=$PT SRNN_SOUP_LANES=2 SRNN_X2_EMULATE_REMOTE=0.164 timeout -k 10 300 python bench.py --steps 20 \
    --warmup 5 --force-sharded --particles 12500 --reference-order-steps 0 > gpurun_out/strong_8_t${PT}_$TAG.log 2>&1 || exit 1
  echo "strong model R=8 table=$PT: $(tail -1 gpurun_out/strong_8_t${PT}_$TAG.log | cut -c1-200)"
done
