#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export MASTER_ADDR=127.0.0.1
for m in release_destroy release_none none; do
SRNN_REHEARSAL_EXIT=$m MASTER_PORT=$((29570 + ${#m})) timeout -k 10 60 python -u bench/sharded_rehearsal.py --n 20000 --gens 5 > gpurun_out/rh_$m.log 2>&1; rc=$?; echo "$m rc=$rc"; grep rehearsal gpurun_out/rh_$m.log | tail -3
if [ $rc -ne 0 ]; then exit $rc; fi
done
