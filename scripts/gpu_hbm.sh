#!/bin/bash
# BASELINE config 5 on one MI355X: sharded (all-to-all) layout forced at one rank above 2^31 slots,
# HBM-filling, with a streaming checkpoint round trip.  Small dry run first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CK=${TMPDIR}/srnn_hbm_ck
df -h $TMPDIR . > gpurun_out/hbm_df.log 2>&1
free -g >> gpurun_out/hbm_df.log 2>&1
timeout -k 10 300 python -u bench/hbm_soup.py --n 20000000 --gens 3 --sharded --checkpoint $CK > gpurun_out/hbm_small.log 2>&1 && tail -2 gpurun_out/hbm_small.log &&
timeout -k 10 1000 python -u bench/hbm_soup.py --gens 3 --sharded --checkpoint $CK > gpurun_out/hbm_big.log 2>&1; rc=$?
tail -3 gpurun_out/hbm_big.log; rm -rf $CK; exit $rc
