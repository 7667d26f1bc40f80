#!/bin/bash
# Headline bench only: K=20 (driver form) twice, K=50, and a kernel-stats profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-bench}
for k in 20 20 50; do
  timeout -k 10 300 python bench.py --steps $k --warmup 5 > gpurun_out/${TAG}_$k.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('K', sys.argv[2], d['ms_per_step'])" gpurun_out/${TAG}_$k.log $k
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o b --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_$TAG.log 2>&1 &&
python -c "
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:3]: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,2))" gpurun_out/prof_$TAG/b_kernel_stats.csv
