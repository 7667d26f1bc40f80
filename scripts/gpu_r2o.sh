#!/bin/bash
# r2o: multi-generation graph sizes for the driver's 20-generation timed window (16 + 4 vs one
# 20-generation graph), alternated A/B/A/B on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ms() { grep -o '"ms_per_step": [0-9.]*' "$1"; }
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/o_a$k.log 2>&1 && echo -n "chunks 16,8,4,2 K=20: " && ms gpurun_out/o_a$k.log &&
  SRNN_GRAPH_CHUNKS=20,16,8,4,2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/o_b$k.log 2>&1 && echo -n "chunks 20,16,8,4,2 K=20: " && ms gpurun_out/o_b$k.log || exit 1
done
