#!/bin/bash
# The reference's published experiments (code/results/**/log.txt) re-run at 100-10000x their
# trial counts on one MI355X (setups CLI, device cuda): one JSON line per experiment.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/parity.jsonl
: > $OUT
run() {
  local name=$1; shift
  local t0=$(date +%s.%N)
  timeout -k 10 240 python -u -m self_replicating_neural_networks_amd.setups $name --device cuda --root $TMPDIR/exps "$@" > gpurun_out/parity_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/parity_$name.log; return 1; }
  local t1=$(date +%s.%N)
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); d.pop('dir',None); d['experiment']=sys.argv[2]; d['args']=sys.argv[4:]; d['seconds']=round(float(sys.argv[3]),1); print(json.dumps(d))" gpurun_out/parity_$name.log $name $(python -c "import sys; print(float(sys.argv[2])-float(sys.argv[1]))" $t0 $t1) "$@" >> $OUT
  echo "$name done"
}
run applying_fixpoints --trials 200000 &&
run training_fixpoints --trials 20000 &&
run known_fixpoint_variation --trials 100000 &&
run learn_from_soup --trials 2000 &&
run mixed_soup --trials 2000 &&
run mixed_self_fixpoints --trials 2000
