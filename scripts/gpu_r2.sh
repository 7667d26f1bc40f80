#!/bin/bash
# Round-2 GPU check: GPU tests (per-test timeout), smoke, headline bench, kernel-trace profile.
# Every GPU step has its own time limit; a fault / abort / timeout stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2}
SEL=${2:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread $SEL > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 && cat gpurun_out/bench_$TAG.log
