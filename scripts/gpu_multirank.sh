#!/bin/bash
# Rehearse the sharded soup on ONE GPU: 2 ranks sharing cuda:0 (gloo, then RCCL).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 --share-device --backend gloo > gpurun_out/mr_gloo.log 2>&1; rc=$?; echo "gloo rc=$rc"; grep metric gpurun_out/mr_gloo.log | cut -c1-250
if [ $rc -gt 1 ] && [ $rc -ne 124 ]; then tail -5 gpurun_out/mr_gloo.log; fi
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 2 --share-device > gpurun_out/mr_nccl.log 2>&1; echo "nccl rc=$?"; grep -E "metric|Error|error" gpurun_out/mr_nccl.log | head -5 | cut -c1-300
