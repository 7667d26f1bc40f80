#!/bin/bash
# Lean closing check: every GPU test, smoke(), then the headline A/B against ab_base/ (same box,
# alternated) and one headline run with the reference-order side measurement.
#   bash scripts/gpu_closing2.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-c2}
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" gpurun_out/pytest_$TAG.log | head -20; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
echo "smoke ok"
for i in 1 2; do
  for V in base new; do
    D=.; [ $V = base ] && D=ab_base
    (cd $D && timeout -k 10 300 python bench.py --steps 20 --warmup 5) > gpurun_out/abx_${V}_${i}_$TAG.log 2>&1 || exit 1
    echo "$V $i: $(tail -1 gpurun_out/abx_${V}_${i}_$TAG.log | cut -c150-200)"
  done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --reference-order-steps 20 > gpurun_out/bench_ro_$TAG.log 2>&1 || exit 1
echo "ro: $(tail -1 gpurun_out/bench_ro_$TAG.log | grep -o '"reference_order": {"steps": 20, "ms_per_step": [0-9.]*')"
