#!/bin/bash
# Kernel traces of the forced-sharded (one-rank RCCL all-to-all pipeline) and unsharded benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-prof}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fs_$TAG -o fs --output-format csv -- python3 bench.py --steps 20 --warmup 3 --force-sharded > gpurun_out/prof_fs_$TAG.log 2>&1 && echo "prof fs ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_1_$TAG -o one --output-format csv -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/prof_1_$TAG.log 2>&1 && echo "prof 1 ok"
