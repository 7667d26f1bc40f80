#!/bin/bash
# Quick GPU iteration: selected GPU tests, headline bench, kernel-trace stats of the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-q}
SEL=${2:-soup}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$SEL" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 5 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 200 --warmup 10 > gpurun_out/bench_$TAG.log 2>&1 && cat gpurun_out/bench_$TAG.log | grep metric &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o bench --output-format csv -- python bench.py --steps 40 --warmup 3 > gpurun_out/prof_$TAG.log 2>&1 &&
for f in $(find gpurun_out/prof_$TAG -name "*kernel_stats.csv"); do python scripts/prof_summary.py $f; done
