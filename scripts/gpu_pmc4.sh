#!/bin/bash
# Counter passes (one --pmc run each, kernel-trace only) of the WW(2,2) generation kernels:
# one lane per particle (k_soup_gen) vs a lane pair (k_soup_gen2) at 100k and 12.5k particles,
# permutation table off (the inline draws) and on.
#   bash scripts/gpu_pmc4.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4p}
C1="SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU"
C2="SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
for N in 100000 12500; do
  for L in 1 2; do
    for PT in 0 1; do
      for P in 1 2; do
        CS=$C1; [ $P = 2 ] && CS=$C2
        SRNN_SOUP_LANES=$L SRNN_PERM_TABLE=$PT timeout -s KILL 90 rocprofv3 --pmc $CS -d gpurun_out/pmc4_${N}_${L}_${PT}_${P}_$TAG \
          -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-graph --particles $N \
          --reference-order-steps 0 > gpurun_out/pmc4_${N}_${L}_${PT}_${P}_$TAG.log 2>&1 || exit 1
      done
      echo "pmc n=$N lanes=$L table=$PT ok"
    done
  done
done
