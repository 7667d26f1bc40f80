#!/bin/bash
# GPU tests + forced-sharded bench + kernel trace of the forced-sharded and unsharded benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3c}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --force-sharded > gpurun_out/benchfs_$TAG.log 2>&1 && tail -1 gpurun_out/benchfs_$TAG.log | cut -c1-300 &&
SRNN_LOOPBACK=1 timeout -k 10 300 python bench.py --steps 50 --warmup 5 --force-sharded > gpurun_out/benchlb_$TAG.log 2>&1 && tail -1 gpurun_out/benchlb_$TAG.log | cut -c1-300 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fs_$TAG -o fs --output-format csv -- python3 bench.py --steps 20 --warmup 3 --force-sharded > gpurun_out/prof_fs_$TAG.log 2>&1 && echo "prof fs ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_1_$TAG -o one --output-format csv -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/prof_1_$TAG.log 2>&1 && echo "prof 1 ok"
