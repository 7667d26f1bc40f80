#!/bin/bash
# The current measurement sequence (edited as the work moves on; the record of what each run
# measured is its profiles/r*.md).  Every GPU step has its own time limit; the first failure
# that is not a test failure stops the script.
#   bash scripts/gpu_round.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-round}
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/${name}_$TAG.log 2>&1; local rc=$?;
         echo "[$name rc=$rc] $(tail -1 gpurun_out/${name}_$TAG.log | cut -c1-600)"; return $rc; }
timeout -k 10 600 python -u -m pytest tests/test_sharded_multirank_gpu.py tests/test_sharded_gpu.py tests/test_bench_contract_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
# strong-scaling model of one rank of N (forced-sharded, remote fraction emulated), kernel traces
for NR in 8:12500:0.164 4:25000:0.141 2:50000:0.093; do
  IFS=: read R NP FR <<< "$NR"
  SRNN_X2_EMULATE_REMOTE=$FR step xprof${R} 300 rocprofv3 --kernel-trace --stats -d gpurun_out/xprof${R}_$TAG -o x --output-format csv -- python3 bench.py --steps 20 --warmup 5 --force-sharded --particles $NP --reference-order-steps 0 || exit 1
  SRNN_X2_EMULATE_REMOTE=$FR step strong${R} 300 python bench.py --steps 20 --warmup 5 --force-sharded --particles $NP --reference-order-steps 0 || exit 1
  SRNN_X2_EMULATE_REMOTE=$FR step strong${R}b 300 python bench.py --steps 20 --warmup 5 --force-sharded --particles $NP --reference-order-steps 0 || exit 1
done
step b20 300 python bench.py --steps 20 --warmup 5 || exit 1
echo done
