#!/bin/bash
# Sharded-generation breakdown: kernel traces of the forced-sharded 8-rank model at one rank
# (12.5k slots, 16.4 % remote) and of the 2-rank model (50k slots), plus the multi-rank GPU tests.
#   bash scripts/gpu_r4d.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4d}
timeout -k 10 400 python -u -m pytest tests/test_sharded_gpu.py tests/test_sharded_multirank_gpu.py -m gpu --maxfail=4 -v \
  --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/pytest_$TAG.log | tail -3
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" gpurun_out/pytest_$TAG.log | head -20; exit $rc; fi
for NR in 8:12500:0.164 2:50000:0.093; do
  IFS=: read R NP FR <<< "$NR"
  SRNN_X2_EMULATE_REMOTE=$FR timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/xprof_${R}_$TAG -o x \
    --output-format csv -- python3 bench.py --steps 20 --warmup 5 --force-sharded --particles $NP \
    --reference-order-steps 0 > gpurun_out/xprof_${R}_$TAG.log 2>&1 || exit 1
  echo "R=$R: $(tail -1 gpurun_out/xprof_${R}_$TAG.log | cut -c1-160)"
done
