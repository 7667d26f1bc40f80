#!/bin/bash
# r2j: coalesced (LDS-staged) row transfers of the big-net kernels + one-workgroup-per-generation
# batched finish: full GPU suite, headline bench at the driver's K=20 and at 200 steps, config 4
# and the Aggregating(4,10,3) soup, kernel traces of both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pt_r2j.log 2>&1
rc=$?; tail -5 gpurun_out/pt_r2j.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$k.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench20_$k.log').read().strip().splitlines()[-1]); print('K=20', d['ms_per_step'])"
done
timeout -k 10 300 python bench.py --steps 200 --warmup 10 > gpurun_out/bench200.log 2>&1 &&
python -c "import json; d=json.loads(open('gpurun_out/bench200.log').read().strip().splitlines()[-1]); print('K=200', d['ms_per_step'])" &&
timeout -k 10 600 python bench/configs.py --only 4,4s > gpurun_out/cfg4.jsonl 2> gpurun_out/cfg4.err && cat gpurun_out/cfg4.jsonl &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2j -o cfg --output-format csv -- python bench/configs.py --only 4,4s --reps 3 --n4s 200000 --gens4s 3 > gpurun_out/prof_r2j.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2j_b -o bench --output-format csv -- python bench.py --steps 20 --warmup 3 > gpurun_out/prof_r2j_b.log 2>&1 &&
for f in $(find gpurun_out/prof_r2j gpurun_out/prof_r2j_b -name "*kernel_stats.csv"); do python scripts/prof_summary.py $f | head -24; done
