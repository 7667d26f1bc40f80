#!/bin/bash
# Round-3 GPU check: GPU tests, smoke, 1-GPU bench, the sharded all-to-all pipeline forced at
# one rank (RCCL + graphs) and at 2 ranks sharing the card (gloo), bench self-launch.
# Every GPU step has its own timeout; anything but a test failure (rc 1) stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1_$TAG.log 2>&1 && tail -1 gpurun_out/bench1_$TAG.log &&
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench1b_$TAG.log 2>&1 && tail -1 gpurun_out/bench1b_$TAG.log &&
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --force-sharded > gpurun_out/benchfs_$TAG.log 2>&1 && tail -1 gpurun_out/benchfs_$TAG.log &&
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 --share-device --backend gloo > gpurun_out/bench2_$TAG.log 2>&1 && tail -1 gpurun_out/bench2_$TAG.log
