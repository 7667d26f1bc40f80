#!/bin/bash
# Quick GPU pass: selected test files (default: the exact-oracle and ordered tests), smoke(),
# one driver-form bench.  Every step has its own timeout; the script stops at the first
# non-test failure.
#   bash scripts/gpu_quick.sh <tag> [test files...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-quick}; shift
TESTS=${*:-tests/test_exact_oracle_gpu.py tests/test_ordered_soup.py}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_$TAG.log | head -20; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$TAG.log 2>&1 && tail -1 gpurun_out/bench20_$TAG.log | cut -c1-400
