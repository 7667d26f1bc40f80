#!/bin/bash
# r2l: self-closing sharded generation (in-kernel pack + last-wave stats, SRNN_GEN_PACK) vs the
# finish-launch pipeline: full GPU suite (incl. 2/3-rank device soups), forced-sharded bench A/B,
# 2-rank gloo shared-device bench, kernel trace of the forced-sharded run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pt_r2l.log 2>&1; rc=$?; tail -3 gpurun_out/pt_r2l.log; [ $rc -eq 0 ] || exit $rc
ms() { grep -o '"ms_per_step": [0-9.]*' "$1"; }
timeout -k 10 300 python bench.py --steps 200 --warmup 10 > gpurun_out/l_single.log 2>&1 && echo -n "single: " && ms gpurun_out/l_single.log &&
for k in 1 2; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 10 --force-sharded > gpurun_out/l_pack_$k.log 2>&1 && echo -n "sharded gen_pack: " && ms gpurun_out/l_pack_$k.log &&
  SRNN_GEN_PACK=0 timeout -k 10 300 python bench.py --steps 200 --warmup 10 --force-sharded > gpurun_out/l_fin_$k.log 2>&1 && echo -n "sharded finish: " && ms gpurun_out/l_fin_$k.log || exit 1
done &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force-sharded > gpurun_out/l_pack20.log 2>&1 && echo -n "sharded gen_pack K=20: " && ms gpurun_out/l_pack20.log &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 20 --warmup 2 --share-device --backend gloo > gpurun_out/l_2rank.log 2>&1 && echo -n "2 gloo ranks: " && ms gpurun_out/l_2rank.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_l -o sh --output-format csv -- python bench.py --steps 40 --warmup 3 --force-sharded > gpurun_out/prof_l.log 2>&1 &&
for f in $(find gpurun_out/prof_l -name "*kernel_stats.csv"); do python scripts/prof_summary.py $f > gpurun_out/prof_l_summary.md; head -12 gpurun_out/prof_l_summary.md; done
