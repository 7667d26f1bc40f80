#!/bin/bash
# Train / soup timings of the reference's other shapes (bench/shape_bench.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-shapes}
timeout -k 10 900 python -u bench/shape_bench.py ${@:2} > gpurun_out/${TAG}.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/${TAG}.log | tail -12; exit $rc
