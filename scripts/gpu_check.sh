#!/bin/bash
# GPU check: tests, smoke, bench (+ optional profile). Each GPU step has its own timeout;
# test failures (rc 1) do not stop the script, anything else (fault/abort/timeout) does.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 && cat gpurun_out/bench_$TAG.log &&
timeout -k 10 300 python bench/kernel_bench.py --only "weightwise(0,2,2" > gpurun_out/kbench_$TAG.log 2>&1 && cat gpurun_out/kbench_$TAG.log | grep arch &&
if [ "$2" == "prof" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o bench --output-format csv -- python bench.py --steps 20 --warmup 3 > gpurun_out/prof_$TAG.log 2>&1 && echo "prof ok"
fi
