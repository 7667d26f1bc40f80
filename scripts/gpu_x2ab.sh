#!/bin/bash
# Sharded-pipeline check + A/B at one rank: device sharded tests, forced-sharded bench with RCCL
# and with the one-rank loopback copy, and the timing model of 8 ranks (16.4 % of the slots
# through the remote list after the exchange), with a kernel trace of the model.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-x2ab}
B="python bench.py --steps 50 --warmup 5 --force-sharded"
run() { # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 $B > gpurun_out/${TAG}_$name.log 2>&1 || return $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" gpurun_out/${TAG}_$name.log $name
}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sharded_multirank_gpu.py tests/test_bench_contract_gpu.py > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 50 --warmup 5 > gpurun_out/${TAG}_plain.log 2>&1 && tail -1 gpurun_out/${TAG}_plain.log | cut -c1-200 &&
run fs_ser SRNN_X2_SCHEDULE=serial && run fsl_ser SRNN_X2_SCHEDULE=serial SRNN_LOOPBACK=1 &&
run fsl_ovl SRNN_X2_SCHEDULE=overlap SRNN_LOOPBACK=1 &&
run em_ser SRNN_X2_SCHEDULE=serial SRNN_X2_EMULATE_REMOTE=0.164 && run eml_ser SRNN_X2_SCHEDULE=serial SRNN_LOOPBACK=1 SRNN_X2_EMULATE_REMOTE=0.164 &&
run eml_ovl SRNN_X2_SCHEDULE=overlap SRNN_LOOPBACK=1 SRNN_X2_EMULATE_REMOTE=0.164 &&
SRNN_X2_SCHEDULE=serial SRNN_LOOPBACK=1 SRNN_X2_EMULATE_REMOTE=0.164 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_emul_$TAG -o emul --output-format csv -- python3 bench.py --steps 20 --warmup 3 --force-sharded > gpurun_out/prof_emul_$TAG.log 2>&1 && echo "prof emul ok"
