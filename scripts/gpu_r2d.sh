#!/bin/bash
# r2d: big-net row kernels (all storage formats / shufflers) vs the runtime-shape engine, the
# Aggregating(4,10,3) soup config, full GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pt_big.log 2>&1
rc=$?; tail -25 gpurun_out/pt_big.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 900 python bench/configs.py --only 4s > gpurun_out/cfg4s.jsonl 2> gpurun_out/cfg4s.err && cat gpurun_out/cfg4s.jsonl &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_4s -o p4s --output-format csv -- python bench/configs.py --only 4s --n4s 200000 --gens4s 3 > gpurun_out/prof_4s.log 2>&1 &&
for f in $(find gpurun_out/prof_4s -name "*kernel_stats.csv"); do python scripts/prof_summary.py $f | head -24; done
