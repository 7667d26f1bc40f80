#!/bin/bash
# Full GPU check: every GPU test, smoke(), the 1-GPU bench in the driver's form (K=20, twice) and
# at K=50, the forced-sharded bench (the multi-GPU protocol at one rank), the self-launched
# 2-rank bench (gloo, ranks sharing the card), and a kernel trace of the K=20 bench.
# Every GPU step has its own timeout; anything but a test failure stops the script.
#   bash scripts/gpu_check.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-check}
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log
# test failures (rc 1) are listed and the rest still runs; a fault / abort / timeout stops it
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" gpurun_out/pytest_$TAG.log | head -20; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$TAG.log 2>&1 && tail -1 gpurun_out/bench20_$TAG.log | cut -c1-250 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20b_$TAG.log 2>&1 && tail -1 gpurun_out/bench20b_$TAG.log | cut -c1-250 &&
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench50_$TAG.log 2>&1 && tail -1 gpurun_out/bench50_$TAG.log | cut -c1-250 &&
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --force-sharded > gpurun_out/benchfs_$TAG.log 2>&1 && tail -1 gpurun_out/benchfs_$TAG.log | cut -c1-250 &&
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 --share-device --backend gloo > gpurun_out/bench2_$TAG.log 2>&1 && tail -1 gpurun_out/bench2_$TAG.log | cut -c1-250 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o b20 --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_$TAG.log 2>&1 && echo "prof ok"
