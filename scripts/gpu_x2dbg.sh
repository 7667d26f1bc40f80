#!/bin/bash
# Sharded pipeline forced at one rank, stage by stage (eager, then with graphs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -u bench/x2_debug.py 100000 > gpurun_out/x2dbg_eager.log 2>&1; rc=$?
cat gpurun_out/x2dbg_eager.log | grep -v amdgpu.ids | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -u bench/x2_debug.py 100000 --graph > gpurun_out/x2dbg_graph.log 2>&1; rc=$?
cat gpurun_out/x2dbg_graph.log | grep -v amdgpu.ids | tail -30
exit $rc
