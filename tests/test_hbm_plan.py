"""HBM sizing of node-wide soups (BASELINE config 5, "288 GB HBM sizing"): the sharded all-to-all
layout addresses int64 slots with O(local) per-rank state, so an 8-rank soup is limited by HBM,
not by 32-bit list entries (profiles/r3c: 3.1e9 particles in 284 GB on one MI355X)."""
import torch

from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.soup_engine import engine_bytes, plan_population


def test_eight_rank_alltoall_soup_is_hbm_limited():
    p = plan_population(ArchSpec.weightwise(2, 2), torch.float16, exchange="alltoall", world=8)
    assert p["limited_by"] == "hbm"
    assert p["n_total"] > 2 ** 32  # node-wide slots beyond 32 bits
    assert p["bytes_per_gpu"] <= 0.9 * 288e9
    # per-rank memory is O(local): doubling the ranks at a fixed node population halves it
    n = 4 * 10 ** 9
    b8 = engine_bytes(ArchSpec.weightwise(2, 2), n, world=8, dtype=torch.float16)
    b16 = engine_bytes(ArchSpec.weightwise(2, 2), n, world=16, dtype=torch.float16)
    assert 0.45 < b16 / b8 < 0.6


def test_one_rank_sharded_layout_fits_above_2_31():
    p = plan_population(ArchSpec.weightwise(2, 2), torch.float16, exchange="alltoall", world=1)
    assert p["limited_by"] == "hbm" and p["n_total"] > 2 ** 31


def test_allgather_exchange_reports_its_32_bit_limit():
    p = plan_population(ArchSpec.weightwise(2, 2), torch.float16, exchange="allgather", world=8)
    assert p["limited_by"] == "uint32 list entries" and p["n_total_fit"] > p["n_total"]
