#!/bin/bash
# Profiles of one bench configuration (rocprofv3; the counter passes one per run, kernel trace
# only, each under its own hard time limit -- a request beyond the hardware's counters hangs).
#   bash scripts/gpu_prof.sh <tag> trace [bench args...]   kernel trace + stats
#   bash scripts/gpu_prof.sh <tag> pmc [bench args...]     two SQ counter passes (VALU, LDS, waves,
#                                                          wave cycles split into issuing / waiting /
#                                                          issue-stalled, bank conflicts, clock)
# Environment variables on the command line (SRNN_* knobs) select the kernel variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-prof}; MODE=${2:-trace}
shift 2 2>/dev/null || shift $#
ARGS=${*:---steps 20 --warmup 5}
if [ "$MODE" = trace ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o t --output-format csv -- \
    python3 bench.py $ARGS > gpurun_out/prof_$TAG.log 2>&1 && echo "trace $TAG ok"
  exit $?
fi
C1="SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU"
C2="SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
for P in 1 2; do
  CS=$C1; [ $P = 2 ] && CS=$C2
  timeout -s KILL 120 rocprofv3 --pmc $CS -d gpurun_out/pmc_${TAG}_$P -o p --output-format csv -- \
    python3 bench.py $ARGS > gpurun_out/pmc_${TAG}_$P.log 2>&1 || exit 1
  echo "pmc $TAG pass $P ok"
done
