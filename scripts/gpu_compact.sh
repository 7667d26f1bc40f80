#!/bin/bash
# A/B of the heavy-slot compaction in the fused generation + the kernel GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-cmp}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_lowp.py > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  SRNN_SOUP_COMPACT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_$v.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('compact', sys.argv[2], d['ms_per_step'], d['config']['final_census'])" gpurun_out/${TAG}_$v.log $v
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o b --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_$TAG.log 2>&1 &&
python -c "
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:3]: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,2))" gpurun_out/prof_$TAG/b_kernel_stats.csv
