#!/bin/bash
# Rehearse bench.py's multi-rank path on ONE GPU: 2 ranks sharing cuda:0 over gloo (RCCL
# refuses two ranks on one device), plus the one-rank RCCL path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 2 --share-device --backend gloo > gpurun_out/mr_gloo.log 2>&1; rc=$?; echo "gloo 2 ranks rc=$rc"; grep metric gpurun_out/mr_gloo.log | cut -c1-300
if [ $rc -ne 0 ]; then tail -20 gpurun_out/mr_gloo.log; exit $rc; fi
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 1 --steps 30 --warmup 3 --force-sharded > gpurun_out/mr_rccl1.log 2>&1; rc=$?; echo "rccl 1 rank (torchrun) rc=$rc"; grep metric gpurun_out/mr_rccl1.log | cut -c1-300
