#!/bin/bash
# Counter passes of the 1M Aggregating(4,10,3) soup kernels (synchronous fp32 / bf16 and the
# reference order), one SQ pass each: VALU / VMEM instructions, wave cycles, waiting.
#   bash scripts/gpu_pmc_big.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
C1="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"
for O in synchronous sequential; do
  timeout -s KILL 300 rocprofv3 --pmc $C1 -d gpurun_out/pmcbig_${O}_$TAG -o p --output-format csv -- \
    python3 bench/configs.py --only 4s --n4s 1000000 --gens4s 1 --order4s $O > gpurun_out/pmcbig_${O}_$TAG.log 2>&1 || exit 1
  echo "pmc $O ok"
done
