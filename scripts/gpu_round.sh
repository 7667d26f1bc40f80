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
SRNN_LIB=$PWD/ab/libsrnn_fine.so step hw 200 python bench/ordered_trace.py --slots 36 --gens 3 || exit 1
SRNN_LIB=$PWD/ab/libsrnn_fine.so step hw3k 200 python bench/ordered_trace.py --slots 36 --particles 3000 --gens 4 || exit 1
# same-box A/B of the census on the side stream (1, default) against the census in the close (0)
for i in 1 2; do
  for cs in 1 0; do
    SRNN_ORD_CENSUS_SIDE=$cs step cs${cs}_$i 300 python bench.py --steps 50 --warmup 5 --side-steps 0 || exit 1
  done
done
SRNN_ORD_CENSUS_SIDE=0 step prof0 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof0_$TAG -o t --output-format csv -- python3 bench.py --steps 20 --warmup 5 --side-steps 0 || exit 1
for f in cs1_1 cs0_1 cs1_2 cs0_2; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], '%.4f' % d['ms_per_step'], d['config']['ord_pipeline'])" gpurun_out/${f}_$TAG.log $f; done
echo done
