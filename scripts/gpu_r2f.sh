#!/bin/bash
# r2f: forced-sharded (1-rank RCCL) generation: bench + kernel trace (per-kernel times and gaps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pt_r2f.log 2>&1; rc=$?; tail -3 gpurun_out/pt_r2f.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 400 --warmup 10 > gpurun_out/b_single.log 2>&1 && grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_single.log &&
timeout -k 10 300 python bench.py --steps 400 --warmup 10 --force-sharded > gpurun_out/b_sharded.log 2>&1 && grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_sharded.log &&
SRNN_SHARDED_GRAPH=0 timeout -k 10 300 python bench.py --steps 400 --warmup 10 --force-sharded --no-graph > gpurun_out/b_sharded_eager.log 2>&1 && grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_sharded_eager.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sh -o sh --output-format csv -- python bench.py --steps 40 --warmup 3 --force-sharded > gpurun_out/prof_sh.log 2>&1 &&
for f in $(find gpurun_out/prof_sh -name "*kernel_stats.csv"); do python scripts/prof_summary.py $f | head -14; done
