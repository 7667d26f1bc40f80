#!/bin/bash
# r2e: BASELINE config 5 at HBM scale (one MI355X): fp16 soup filling the HBM, streaming
# checkpoint round trip; first a 200M-particle rehearsal, then the full size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
df -h /tmp . 2>&1 | tail -3; free -g | head -2
timeout -k 10 300 python -u bench/hbm_soup.py --n 200000000 --gens 2 --checkpoint /tmp/srnn_ck_small > gpurun_out/hbm_small.jsonl 2> gpurun_out/hbm_small.err && cat gpurun_out/hbm_small.jsonl &&
timeout -k 10 900 python -u bench/hbm_soup.py --gens 3 ${CK:+--checkpoint /tmp/srnn_ck_full} > gpurun_out/hbm_full.jsonl 2> gpurun_out/hbm_full.err && cat gpurun_out/hbm_full.jsonl
