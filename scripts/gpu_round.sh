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
timeout -k 10 600 python -u -m pytest tests/test_ordered_soup.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
# same-box A/B: the turn waves wait D us before their first turn (the critical root ahead of the bulk)
for i in 1 2; do
  for D in 10 6 14 0; do
    SRNN_ORD_BULK_DELAY=$D step bd${D}_$i 300 python bench.py --steps 50 --warmup 5 --side-steps 0 || exit 1
  done
done
SRNN_ORD_BULK_DELAY=10 step tr10 200 python bench/ordered_trace.py --gens 2 || exit 1
for f in bd10_1 bd6_1 bd14_1 bd0_1 bd10_2 bd6_2 bd14_2 bd0_2; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], '%.4f' % d['ms_per_step'], d['config']['final_census'])" gpurun_out/${f}_$TAG.log $f; done
echo done
