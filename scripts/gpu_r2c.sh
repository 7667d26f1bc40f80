#!/bin/bash
# r2c: MFMA-vs-VALU micro-benchmark (time + counters per kernel) and the Aggregating(4,10,3) soup config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
C1="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -k 10 120 ./bench/micro/mfma_vs_valu > gpurun_out/mfma_vs_valu.jsonl 2>&1 && cat gpurun_out/mfma_vs_valu.jsonl &&
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc $C1 -d gpurun_out/pmc_mfma -o mv --output-format csv -- ./bench/micro/mfma_vs_valu 100000 1000000 100 > gpurun_out/pmc_mfma.log 2>&1 && echo "pmc ok" &&
timeout -k 10 900 python bench/configs.py --only 4s > gpurun_out/cfg4s.jsonl 2> gpurun_out/cfg4s.err && cat gpurun_out/cfg4s.jsonl
