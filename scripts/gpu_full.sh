#!/bin/bash
# One gpurun call: GPU tests, smoke, headline bench, BASELINE configs, kernel micro-bench,
# kernel-trace profile of the headline bench.  Each GPU step has its own timeout; test
# failures (rc 1) do not stop the script, anything else (fault, abort, timeout) does.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log &&
timeout -k 10 600 python bench/configs.py ${CFG_ONLY:+--only $CFG_ONLY} > gpurun_out/configs.jsonl 2> gpurun_out/configs.err && cat gpurun_out/configs.jsonl &&
timeout -k 10 300 python bench/kernel_bench.py > gpurun_out/kbench.log 2>&1 && echo "kbench ok" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python bench.py --steps 20 --warmup 3 > gpurun_out/prof.log 2>&1 && echo "prof ok" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg -o cfg --output-format csv -- python bench/configs.py --only 2,4 --reps 3 > gpurun_out/prof_cfg.log 2>&1 && echo "prof cfg ok"
