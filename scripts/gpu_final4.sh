#!/bin/bash
# Round-4 closing check: every GPU test, smoke(), the headline twice (driver form) with the
# reference-order side measurement, the BASELINE configs 1/2/4, and counter passes of the wide
# Weightwise wave kernels (register vs LDS SGD: VALU, LDS, waits).
#   bash scripts/gpu_final4.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-f4}
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" gpurun_out/pytest_$TAG.log | head -20; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
echo "smoke ok"
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --reference-order-steps 20 > gpurun_out/bench_${i}_$TAG.log 2>&1 || exit 1
  echo "bench $i: $(tail -1 gpurun_out/bench_${i}_$TAG.log | cut -c150-200)"
done
timeout -k 10 400 python bench/configs.py --only 1,2,4 > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err || exit 1
echo "configs ok"
C1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT"
for W in 1 2; do
  SRNN_WW_WAVE=$W timeout -s KILL 120 rocprofv3 --pmc $C1 -d gpurun_out/pmcww_${W}_$TAG -o p --output-format csv -- \
    python3 bench/shape_bench.py --only "weightwise(10,3)" --reps 1 > gpurun_out/pmcww_${W}_$TAG.log 2>&1 || exit 1
  echo "pmc ww_wave=$W ok"
done
