#!/bin/bash
# GPU tests + the BASELINE.json configs + headline bench (one gpurun call)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pt_cfg.log 2>&1
rc=$?; tail -5 gpurun_out/pt_cfg.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench/configs.py ${CFG_ONLY:+--only $CFG_ONLY} > gpurun_out/configs.jsonl 2> gpurun_out/configs.err && cat gpurun_out/configs.jsonl &&
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench_cfg.log 2>&1 && tail -1 gpurun_out/bench_cfg.log
