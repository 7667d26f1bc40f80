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
# same-box A/B: local hand-offs before the release (default) / release before every hand-off
for i in 1 2 3; do
  step d1_$i 300 python bench.py --steps 50 --warmup 5 --side-steps 0 || exit 1
  SRNN_ORD_DEFER=0 step d0_$i 300 python bench.py --steps 50 --warmup 5 --side-steps 0 || exit 1
done
step tr 200 python bench/ordered_trace.py --gens 2 || exit 1
SRNN_ORD_DEFER=0 step tr0 200 python bench/ordered_trace.py --gens 2 || exit 1
for f in d1_1 d0_1 d1_2 d0_2 d1_3 d0_3; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], '%.4f' % d['ms_per_step'], d['config']['execution']['library']['ord_defer'], d['config']['final_census'])" gpurun_out/${f}_$TAG.log $f; done
echo done
