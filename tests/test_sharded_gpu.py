"""The multi-GPU soup generation on the real device: a one-rank RCCL group drives the
sharded path (row exchange + stats rows through ``all_to_all_single``), eagerly and inside
captured hipGraphs, and must equal the unsharded engine bitwise (bench/sharded_rehearsal.py
in a child process: the process group must not leak into the other tests)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_sharded_path_rccl_graph_equals_unsharded(cuda):
    env = dict(os.environ, SRNN_FORCE_SHARDED="1", MASTER_ADDR="127.0.0.1", MASTER_PORT="29541")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench", "sharded_rehearsal.py"), "--n", "20000",
                        "--gens", "6"], env=env, capture_output=True, text=True, timeout=240)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, p.stdout[-2000:] + p.stderr[-4000:]
    res = json.loads(lines[-1])
    assert res["eager_bitwise_equal"], res
    assert res["graph_bitwise_equal"], res
    assert res["census_equal"], res
    assert res["sharded_graph_captured"], (res, p.stderr[-3000:])
