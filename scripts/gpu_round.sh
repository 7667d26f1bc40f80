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
         echo "[$name rc=$rc] $(tail -1 gpurun_out/${name}_$TAG.log | cut -c1-200)"; return $rc; }
timeout -k 10 600 python -u -m pytest tests/test_ordered_soup.py tests/test_ordered_bignet_gpu.py tests/test_exact_oracle_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
step b1 300 python bench.py --steps 20 --warmup 5 || exit 1
step b2 300 python bench.py --steps 50 --warmup 5 --side-steps 0 || exit 1
echo done
