#!/bin/bash
# GPU tests + counters: MFMA utilisation of the wide Weightwise kernels, VALU/LDS counters of
# the soup generation, roctx ranges of the native ops in a marker trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 250 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc_wide -o wide --output-format csv -- python3 bench/kernel_bench.py --only "weightwise(0,16" --reps 2 > gpurun_out/pmc_wide.log 2>&1 && echo "pmc wide ok" &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc_soup -o soup --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-graph > gpurun_out/pmc_soup.log 2>&1 && echo "pmc soup ok" &&
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU -d gpurun_out/pmc_soup2 -o soup2 --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-graph > gpurun_out/pmc_soup2.log 2>&1 && echo "pmc soup2 ok" &&
SRNN_ROCTX=1 timeout -k 10 120 rocprofv3 --marker-trace --kernel-trace --stats -d gpurun_out/roctx -o rt --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-graph > gpurun_out/roctx.log 2>&1 && echo "roctx ok"
