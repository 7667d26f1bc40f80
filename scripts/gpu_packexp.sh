#!/bin/bash
# Timing experiment: pack with its finish role or its decision role removed (wrong results),
# forced-sharded serial schedule with the 8-rank model, kernel stats per library build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp SRNN_LOOPBACK=1 SRNN_X2_EMULATE_REMOTE=0.164
for v in base NOFINISH NODECIDE; do
  if [ $v = base ]; then unset SRNN_LIB; else export SRNN_LIB=$PWD/exp_libs/libsrnn_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pexp_$v -o p --output-format csv -- python3 bench.py --steps 20 --warmup 3 --force-sharded > gpurun_out/pexp_$v.log 2>&1 || exit $?
  python -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'x2_' in r['Name'] or 'soup_evolve' in r['Name']: print(sys.argv[2], r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,2))" gpurun_out/pexp_$v/p_kernel_stats.csv $v
done
