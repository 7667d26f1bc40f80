#!/bin/bash
# Same-box A/B of the headline (box-to-box spread is up to ~12 %, so builds are only compared
# inside one call): a baseline directory holding bench.py + the package + its libsrnn.so (e.g.
# `git worktree add ab_base <commit>` plus its built library) against this tree, alternated,
# in the driver's form.  Extra arguments go to both bench runs; environment variables set on
# the command line (SRNN_* knobs) apply to both.
#   bash scripts/gpu_ab.sh <tag> <baseline dir> [reps] [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ab}; BASE=${2:-ab_base}; REPS=${3:-3}
shift 3 2>/dev/null || shift $#
ARGS=${*:---steps 20 --warmup 5}
for i in $(seq 1 $REPS); do
  for V in base new; do
    D=.; [ $V = base ] && D=$BASE
    (cd $D && timeout -k 10 300 python bench.py $ARGS) > gpurun_out/ab_${V}_${i}_$TAG.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); ro=d['config'].get('reference_order') or {}; print(sys.argv[2], sys.argv[3], 'ms/gen %.4f' % d['ms_per_step'], 'reference order %s' % (('%.4f' % ro['ms_per_step']) if ro else '-'))" gpurun_out/ab_${V}_${i}_$TAG.log $V $i
  done
done
