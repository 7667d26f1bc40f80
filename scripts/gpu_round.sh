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
# same-box A/B of the shadow threshold with the bulk delay in force (default 12 us)
for i in 1 2 3; do
  for SH in 32 16 24; do
    SRNN_ORD_SHADOW=$SH step s${SH}_$i 300 python bench.py --steps 50 --warmup 5 --side-steps 0 || exit 1
  done
done
for f in s32_1 s16_1 s24_1 s32_2 s16_2 s24_2 s32_3 s16_3 s24_3; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], '%.4f' % d['ms_per_step'])" gpurun_out/${f}_$TAG.log $f; done
echo done
