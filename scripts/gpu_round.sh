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
timeout -k 10 600 python -u -m pytest tests/test_ordered_sharded_gpu.py tests/test_sharded_multirank_gpu.py tests/test_ordered_soup.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  step fs1_$i 300 python bench.py --steps 20 --warmup 3 --force-sharded --side-steps 0 || exit 1
  SRNN_ORD_PIPELINE=off step fs0_$i 300 python bench.py --steps 20 --warmup 3 --force-sharded --side-steps 0 || exit 1
done
SRNN_ORDSH_EMULATE=8 step em8 300 python bench.py --steps 20 --warmup 3 --force-sharded --side-steps 0 || exit 1
SRNN_ORDSH_EMULATE=8 SRNN_ORD_PIPELINE=off step em8off 300 python bench.py --steps 20 --warmup 3 --force-sharded --side-steps 0 || exit 1
step b1 300 python bench.py --steps 20 --warmup 5 || exit 1
for f in fs1_1 fs0_1 fs1_2 fs0_2 em8 em8off b1; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], '%.4f' % d['ms_per_step'], d['config'].get('final_census'))" gpurun_out/${f}_$TAG.log $f; done
echo done
