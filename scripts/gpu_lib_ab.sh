#!/bin/bash
# Same-box A/B of two builds of libsrnn.so (compiler flags, scheduling): the lone-chain probe and
# the driver-form bench, alternated, plus the bitwise ordered / oracle tests on the candidate.
#   bash scripts/gpu_lib_ab.sh <tag> <candidate .so> [reps]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-libab}; CAND=${2:-ab/libsrnn_ilp.so}; REPS=${3:-2}
SRNN_LIB=$PWD/$CAND timeout -k 10 600 python -u -m pytest tests/test_ordered_soup.py tests/test_exact_oracle_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for V in base cand; do
  L=""; [ $V = cand ] && L=$PWD/$CAND
  SRNN_LIB=$L timeout -k 10 200 python bench/micro/lone_chain_probe.py > gpurun_out/chain_${V}_$TAG.log 2>&1 || exit 1
  grep '"n": 64,' gpurun_out/chain_${V}_$TAG.log | sed "s/^/$V /"
done
for i in $(seq 1 $REPS); do
  for V in base cand; do
    L=""; [ $V = cand ] && L=$PWD/$CAND
    SRNN_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b_${V}_${i}_$TAG.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); j=d['config'].get('jacobi') or {}; print(sys.argv[2], sys.argv[3], 'ref-order ms/gen %.4f' % d['ms_per_step'], 'jacobi %s' % (('%.4f' % j['ms_per_step']) if j else '-'))" gpurun_out/b_${V}_${i}_$TAG.log $V $i
  done
done
echo done
