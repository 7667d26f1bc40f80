#!/bin/bash
# Round-4 GPU check of the new kernels, then measurements (most important first):
#   1. GPU tests of the reference-order generation, lane pairs, the permutation table, the
#      register-resident wide Weightwise SGD, and the soups they touch (fused, sharded, kernels)
#   2. the 1-GPU headline (driver form, K = 20) with its reference-order side measurement
#   3. strong-scaling model of one rank at N = 2 / 4 / 8, lanes vs pairs
#   4. kernel trace of the headline + reference-order run
#   5. lanes-per-particle sweep over population sizes (both orders)
#   6. shape timings of the wide Weightwise nets (register vs LDS SGD)
# Every GPU step has its own timeout; the script stops at the first failure.
#   bash scripts/gpu_r4.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4}
timeout -k 10 600 python -u -m pytest tests/test_ordered_soup.py tests/test_pair_soup_gpu.py tests/test_ww_wave_gpu.py \
  tests/test_sharded_gpu.py tests/test_sharded_multirank_gpu.py tests/test_kernels_gpu.py -m gpu --maxfail=6 -v \
  --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/pytest_$TAG.log | tail -3
# test failures (rc 1) are reported and the measurements still run; anything else (a fault,
# an abort, a timeout) ends the script
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" gpurun_out/pytest_$TAG.log | head -20; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --reference-order-steps -1 > gpurun_out/bench_$TAG.log 2>&1 || exit 1
tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
# strong-scaling model of one rank at N = 2 / 4 / 8 (100k / N slots, the remote-dependent fraction
# of an N-rank soup emulated at one rank: 1 - exp(-0.1 (N-1)/N) + 0.1 (N-1)/N)
for NR in 2:50000:0.093 4:25000:0.141 8:12500:0.164; do
  IFS=: read R NP FR <<< "$NR"
  for L in 1 2; do
    SRNN_SOUP_LANES=$L SRNN_X2_EMULATE_REMOTE=$FR timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force-sharded \
      --particles $NP --reference-order-steps 0 > gpurun_out/strong_${R}_${L}_$TAG.log 2>&1 || exit 1
    echo "strong model R=$R n=$NP lanes=$L: $(tail -1 gpurun_out/strong_${R}_${L}_$TAG.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o sync --output-format csv -- python3 bench.py \
  --steps 20 --warmup 5 --reference-order-steps 20 > gpurun_out/prof_$TAG.log 2>&1 || exit 1
echo "prof ok"
timeout -k 10 420 python -u bench/pair_sweep.py > gpurun_out/pairs_$TAG.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/pairs_$TAG.log | cut -c1-160
for S in "weightwise(3,3)" "weightwise(10,3)" "weightwise(16,2)"; do
  timeout -k 10 300 python -u bench/shape_bench.py --only "$S" >> gpurun_out/shapes_reg_$TAG.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/shapes_reg_$TAG.log | cut -c1-300
SRNN_WW_WAVE=2 timeout -k 10 300 python -u bench/shape_bench.py --only "weightwise(10,3)" > gpurun_out/shapes_lds_$TAG.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/shapes_lds_$TAG.log | cut -c1-300
