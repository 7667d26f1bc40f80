#!/bin/bash
# Round-3 counter passes (one --pmc run each, kernel trace only): the single-launch sharded
# generation in the 8-rank model (k_soup_evolve with fused post, k_x2_pack) and the
# lanes-per-particle Weightwise kernels (k_ww_wave, k_ww_wave_soup).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
C1="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
C2="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU"
for c in 1 2; do
  eval CS=\$C$c
  SRNN_LOOPBACK=1 SRNN_X2_EMULATE_REMOTE=0.164 timeout -s KILL 90 rocprofv3 --pmc $CS -d gpurun_out/pmc3_x2_$c -o x2 --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-graph --force-sharded > gpurun_out/pmc3_x2_$c.log 2>&1 && echo "pmc x2 $c ok" || exit $?
  timeout -s KILL 120 rocprofv3 --pmc $CS -d gpurun_out/pmc3_ww_$c -o ww --output-format csv -- python3 bench/shape_bench.py --only "weightwise(16,2)" --n 16384 --epochs 2 --reps 1 > gpurun_out/pmc3_ww_$c.log 2>&1 && echo "pmc ww $c ok" || exit $?
done
