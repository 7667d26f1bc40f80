#!/bin/bash
# Sharded-path rehearsal on one GPU (one-rank RCCL group): GPU tests, per-generation
# timings eager vs hipGraph-captured collectives, forced-sharded headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 250 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
SRNN_FORCE_SHARDED=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29551 timeout -k 10 300 python bench/sharded_rehearsal.py --n 100000 --gens 30 > gpurun_out/rehearsal.log 2>&1; rc=$?; tail -3 gpurun_out/rehearsal.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
MASTER_ADDR=127.0.0.1 MASTER_PORT=29552 timeout -k 10 300 python bench.py --steps 50 --warmup 5 --force-sharded > gpurun_out/bench_forced.log 2>&1 && tail -1 gpurun_out/bench_forced.log | cut -c1-400 &&
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-300
