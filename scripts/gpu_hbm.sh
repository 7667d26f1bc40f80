#!/bin/bash
# BASELINE config 5 on one MI355X: sharded (all-to-all) layout forced at one rank above 2^31 slots,
# HBM-filling, with a streaming checkpoint round trip (to /dev/shm when it can hold the ~113 GB,
# else to the local disk at the largest population above 2^31 that fits it).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
df -B1 /dev/shm $TMPDIR > gpurun_out/hbm_df.log 2>&1
SHM=$(df -B1 --output=avail /dev/shm 2>/dev/null | tail -1)
if [ -n "$SHM" ] && [ "$SHM" -gt 125000000000 ]; then
  CK=/dev/shm/srnn_hbm_ck; ARGS=""
else
  CK=$TMPDIR/srnn_hbm_ck; ARGS="--n 2160000000"
fi
echo "checkpoint dir $CK $ARGS" | tee -a gpurun_out/hbm_df.log
timeout -k 10 1000 python -u bench/hbm_soup.py --gens 3 --sharded --checkpoint $CK $ARGS > gpurun_out/hbm_big.log 2>&1; rc=$?
tail -3 gpurun_out/hbm_big.log; rm -rf $CK; exit $rc
