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
# one SQ counter pass of eager reference-order generations (no graphs: a counter-collecting profiler
# serialises kernels; the engine's stream probe keeps the side stream's work on events)
C1="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"
timeout -s KILL 150 rocprofv3 --pmc $C1 -d gpurun_out/pmc_$TAG -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --side-steps 0 --no-graph > gpurun_out/pmc_$TAG.log 2>&1 || exit 1
echo "pmc ok"
step b1 300 python bench.py --steps 20 --warmup 5 || exit 1
echo done
