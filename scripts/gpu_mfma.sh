#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pt_mfma.log 2>&1
rc=$?; tail -3 gpurun_out/pt_mfma.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench/kernel_bench.py --only "weightwise(0,16" > gpurun_out/kb_wide.log 2>&1 && grep arch gpurun_out/kb_wide.log &&
timeout -k 10 300 python bench/kernel_bench.py --only "weightwise(0,32" >> gpurun_out/kb_wide.log 2>&1 && grep arch gpurun_out/kb_wide.log | tail -1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_WAVES -d gpurun_out/pmc_wide -o kb --output-format csv -- python bench/kernel_bench.py --only "weightwise(0,16" --reps 2 > gpurun_out/pmc_wide.log 2>&1 && echo pmc ok
