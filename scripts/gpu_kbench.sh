#!/bin/bash
# kernel micro-bench + PMC counters of the soup-evolve path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench/kernel_bench.py > gpurun_out/kbench.log 2>&1 && cat gpurun_out/kbench.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc1 -o kb --output-format csv -- python bench/kernel_bench.py --only weightwise\(0,2,2 --reps 2 > gpurun_out/pmc1.log 2>&1 && echo pmc1 ok &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM -d gpurun_out/pmc2 -o kb --output-format csv -- python bench/kernel_bench.py --only weightwise\(0,2,2 --reps 2 > gpurun_out/pmc2.log 2>&1 && echo pmc2 ok
