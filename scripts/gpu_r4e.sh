#!/bin/bash
# Final measurements: the strong-scaling model of one rank at N = 2 / 4 / 8 (forced-sharded,
# remote fraction emulated) with kernel traces, and counter passes of the wide Weightwise wave
# kernels (register vs LDS SGD).
#   bash scripts/gpu_r4e.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4e2}
for NR in 8:12500:0.164 4:25000:0.141 2:50000:0.093; do
  IFS=: read R NP FR <<< "$NR"
  SRNN_X2_EMULATE_REMOTE=$FR timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/xprof_${R}_$TAG -o x \
    --output-format csv -- python3 bench.py --steps 20 --warmup 5 --force-sharded --particles $NP \
    --reference-order-steps 0 > gpurun_out/xprof_${R}_$TAG.log 2>&1 || exit 1
  SRNN_X2_EMULATE_REMOTE=$FR timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force-sharded --particles $NP \
    --reference-order-steps 0 > gpurun_out/strong_${R}_$TAG.log 2>&1 || exit 1
  echo "R=$R: $(tail -1 gpurun_out/strong_${R}_$TAG.log | cut -c150-200)"
done
C1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT"
for W in 1 2; do
  SRNN_WW_WAVE=$W timeout -s KILL 120 rocprofv3 --pmc $C1 -d gpurun_out/pmcww_${W}_$TAG -o p --output-format csv -- \
    python3 bench/shape_bench.py --only "weightwise(10,3)" --reps 1 > gpurun_out/pmcww_${W}_$TAG.log 2>&1 || exit 1
  echo "pmc ww_wave=$W ok"
done
