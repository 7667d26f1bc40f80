#!/bin/bash
# A/B of two builds of libsrnn.so (compiler flags): headline bench + BASELINE configs 2,4 each.
# usage: gpu_ab_lib.sh <libA> <libB>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in "$@"; do
  tag=$(basename "$L" .so)
  SRNN_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/ab_bench_$tag.log 2>&1 || exit $?
  echo "$tag $(tail -1 gpurun_out/ab_bench_$tag.log)"
  SRNN_LIB=$PWD/$L timeout -k 10 200 python bench/configs.py --only 2,4 --reps 20 > gpurun_out/ab_cfg_$tag.jsonl 2>&1 || exit $?
  echo "$tag"; cat gpurun_out/ab_cfg_$tag.jsonl
done
