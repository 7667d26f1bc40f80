#!/bin/bash
# Counter passes (one --pmc run each, kernel-trace only), BASELINE configs, kernel micro-bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
C1="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
C2="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU"
timeout -s KILL 90 rocprofv3 --pmc $C1 -d gpurun_out/pmc_soup -o soup --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-graph > gpurun_out/pmc_soup.log 2>&1 && echo "pmc soup ok" &&
timeout -s KILL 90 rocprofv3 --pmc $C2 -d gpurun_out/pmc_soup2 -o soup2 --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-graph > gpurun_out/pmc_soup2.log 2>&1 && echo "pmc soup2 ok" &&
timeout -s KILL 90 rocprofv3 --pmc $C1 -d gpurun_out/pmc_wide -o wide --output-format csv -- python3 bench/kernel_bench.py --only "weightwise(0,16" --reps 2 > gpurun_out/pmc_wide.log 2>&1 && echo "pmc wide ok" &&
timeout -s KILL 90 rocprofv3 --pmc $C1 -d gpurun_out/pmc_agg -o agg --output-format csv -- python3 bench/configs.py --only 4 --reps 2 --n4 200000 > gpurun_out/pmc_agg.log 2>&1 && echo "pmc agg ok" &&
timeout -k 10 600 python bench/configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err && echo "configs ok" &&
timeout -k 10 300 python bench/kernel_bench.py > gpurun_out/kbench.log 2>&1 && echo "kbench ok"
