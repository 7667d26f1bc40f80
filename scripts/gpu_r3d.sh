#!/bin/bash
# GPU tests, smoke, 1-GPU bench at K=20 and K=50 (driver form) and a kernel trace of the K=20 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3d}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$TAG.log 2>&1 && tail -1 gpurun_out/bench20_$TAG.log | cut -c1-250 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20b_$TAG.log 2>&1 && tail -1 gpurun_out/bench20b_$TAG.log | cut -c1-250 &&
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench50_$TAG.log 2>&1 && tail -1 gpurun_out/bench50_$TAG.log | cut -c1-250 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o b20 --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_$TAG.log 2>&1 && echo "prof ok"
