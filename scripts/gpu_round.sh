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
         echo "[$name rc=$rc] $(tail -1 gpurun_out/${name}_$TAG.log | cut -c1-300)"; return $rc; }
bj() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); ro=d['config'].get('reference_order') or {}; print(sys.argv[1], 'ms/gen %.4f' % d['ms_per_step'], d['semantics'], 'ref-order %s' % (('%.4f' % ro['ms_per_step']) if ro else '-'), 'levels', (ro or {}).get('levels') or d['config'].get('ordered_levels'))" gpurun_out/$1_$TAG.log; }
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" gpurun_out/pytest_$TAG.log | head -20; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step b20 300 python bench.py --steps 20 --warmup 5 && bj b20 || exit 1
SRNN_ORD_CRIT=0 step b20nocrit 300 python bench.py --steps 20 --warmup 5 && bj b20nocrit || exit 1
step b20again 300 python bench.py --steps 20 --warmup 5 && bj b20again || exit 1
for N in 12500 25000; do
  for PT in 0 1; do
    for L in 1 2; do
      SRNN_PERM_TABLE=$PT SRNN_SOUP_LANES=$L step s${N}_t${PT}_l${L} 300 python bench.py --steps 20 --warmup 5 --particles $N --reference-order-steps 0 && bj s${N}_t${PT}_l${L} || exit 1
    done
  done
done
step prof_ro 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ro_$TAG -o t --output-format csv -- python3 bench.py --steps 20 --warmup 5 --order sequential || exit 1
SRNN_ORD_CRIT=0 step prof_ronc 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ronc_$TAG -o t --output-format csv -- python3 bench.py --steps 20 --warmup 5 --order sequential || exit 1
echo done
