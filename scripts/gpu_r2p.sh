#!/bin/bash
# r2p: refreshed hardware counters for the round-2 kernels (one --pmc pass per run, kernel-trace
# only): headline generation (k_soup_gen + batched finish) and the P = 280 staged row kernels
# (config 4 ops + a 1M-particle soup), incl. HBM bytes (TCC FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
C1="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
C2="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU"
AGG="python3 bench/configs.py --only 4 --reps 2 --n4 1000000 --n4s 1000000 --gens4s 2"
timeout -s KILL 90 rocprofv3 --pmc $C1 -d gpurun_out/p_soup1 -o s1 --output-format csv -- python3 bench.py --steps 20 --warmup 2 > gpurun_out/p_soup1.log 2>&1 && echo "soup c1 ok" &&
timeout -s KILL 90 rocprofv3 --pmc $C2 -d gpurun_out/p_soup2 -o s2 --output-format csv -- python3 bench.py --steps 20 --warmup 2 > gpurun_out/p_soup2.log 2>&1 && echo "soup c2 ok" &&
timeout -s KILL 120 rocprofv3 --pmc $C1 -d gpurun_out/p_agg1 -o a1 --output-format csv -- $AGG > gpurun_out/p_agg1.log 2>&1 && echo "agg c1 ok" &&
timeout -s KILL 120 rocprofv3 --pmc $C2 -d gpurun_out/p_agg2 -o a2 --output-format csv -- $AGG > gpurun_out/p_agg2.log 2>&1 && echo "agg c2 ok" &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum FETCH_SIZE -d gpurun_out/p_agg3 -o a3 --output-format csv -- $AGG > gpurun_out/p_agg3.log 2>&1 && echo "agg fetch ok" &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/p_agg4 -o a4 --output-format csv -- $AGG > gpurun_out/p_agg4.log 2>&1 && echo "agg write ok"
for d in p_soup1 p_soup2 p_agg1 p_agg2 p_agg3 p_agg4; do
  f=$(find gpurun_out/$d -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && python3 scripts/pmc_summary.py "$f" "$d" > gpurun_out/$d.md
done
exit 0
