#!/bin/bash
# The current measurement sequence (edited as the work moves on; the record of what each run
# measured is its profiles/r*.md).  Every GPU step has its own time limit; the first failure
# that is not a test failure stops the script.
#   bash scripts/gpu_round.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-round}
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/${name}_$TAG.log 2>&1; local rc=$?;
         echo "[$name rc=$rc] $(tail -1 gpurun_out/${name}_$TAG.log | cut -c1-200)"; return $rc; }
timeout -k 10 600 python -u -m pytest tests/test_ordered_soup.py tests/test_ordered_bignet_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
# the bulk delay (default 12 us, first residency round only) on the 1M Aggregating(4,10,3) reference-order
# soup and on the 100k bench soup
for i in 1 2; do
  step big12_$i 300 python bench/configs.py --only 4s --order4s sequential --gens4s 5 || exit 1
  SRNN_ORD_BULK_DELAY=0 step big0_$i 300 python bench/configs.py --only 4s --order4s sequential --gens4s 5 || exit 1
  step d12_$i 300 python bench.py --steps 50 --warmup 5 --side-steps 0 || exit 1
  SRNN_ORD_BULK_DELAY=0 step d0_$i 300 python bench.py --steps 50 --warmup 5 --side-steps 0 || exit 1
done
for f in big12_1 big0_1 big12_2 big0_2; do python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], '%.3f %.3f %.3f' % (d['ref_order_fp32_ms_per_generation'], d['ref_order_bf16_ms_per_generation'], d['ref_order_fp32_shuffle_random_ms_per_generation']))" gpurun_out/${f}_$TAG.log $f; done
for f in d12_1 d0_1 d12_2 d0_2; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], '%.4f' % d['ms_per_step'])" gpurun_out/${f}_$TAG.log $f; done
echo done
