#!/bin/bash
# GPU check: tests, smoke, bench, kernel-trace profile. Every GPU step has its own timeout;
# test failures (rc 1) do not stop the script, anything else (fault, abort, timeout) does.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench1.log 2>&1 && cat gpurun_out/bench1.log &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-graph > gpurun_out/bench1_nograph.log 2>&1 && cat gpurun_out/bench1_nograph.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python bench.py --steps 20 --warmup 3 --no-graph > gpurun_out/prof.log 2>&1 && echo "prof ok"
