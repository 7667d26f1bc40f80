#!/bin/bash
# headline bench vs timed steps / warmup (short timed regions)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pt_steps.log 2>&1; rc=$?; tail -1 gpurun_out/pt_steps.log; [ $rc -eq 0 ] || exit $rc
for sw in "20 5" "20 5" "20 50" "50 5" "200 5" "400 10" "20 5"; do
  set -- $sw
  timeout -k 10 120 python bench.py --steps $1 --warmup $2 > gpurun_out/steps.log 2>&1 || { tail -3 gpurun_out/steps.log; exit 1; }
  echo "steps $1 warmup $2: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/steps.log)"
done
