"""ArchSpec: parameter counts, layouts and coordinates (reference code/network.py)."""
import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from self_replicating_neural_networks_amd.arch import ArchSpec, normalize_id


def test_reference_default_sizes():
    assert ArchSpec.weightwise(2, 2).P == 14          # (4,2),(2,2),(2,1)
    assert ArchSpec.aggregating(4, 2, 2).P == 20      # (4,2),(2,2),(2,4)
    assert ArchSpec.recurrent(2, 2).P == 17           # (1,2)+(2,2), (2,2)+(2,2), (2,1)+(1,1)
    assert ArchSpec.aggregating(4, 10, 3).P == 280    # north-star config
    assert ArchSpec.weightwise(2, 2).PP == 16


@settings(max_examples=50, deadline=None)
@given(w=st.integers(1, 12), d=st.integers(1, 5))
def test_param_count_formulas(w, d):
    assert ArchSpec.weightwise(w, d).P == 4 * w + (d - 1) * w * w + w
    assert ArchSpec.recurrent(w, d).P == (w + w * w) + (d - 1) * 2 * w * w + (w + 1)


def test_normalize_id():
    assert normalize_id(0, 0) == 0.0 and normalize_id(1, 1) == 1.0
    assert normalize_id(1, 3) == pytest.approx(1 / 3) and normalize_id(2, 2) == 1.0


def test_coords_match_reference_points():
    spec = ArchSpec.weightwise(2, 2)
    co = spec.coords()
    assert co.shape == (14, 3)
    # layer 0 (4,2): layer id 0/2, cell i/3, position j/1
    assert tuple(co[0]) == (0.0, 0.0, 0.0) and tuple(co[3]) == (0.0, pytest.approx(1 / 3), 1.0)
    # layer 1 (2,2): layer 1/2
    assert co[8][0] == 0.5 and tuple(co[11][1:]) == (1.0, 1.0)
    # layer 2 (2,1): position norm 0 -> raw 0
    assert tuple(co[12]) == (1.0, 0.0, 0.0) and tuple(co[13]) == (1.0, 1.0, 0.0)


def test_chunks_and_invalid_aggregation():
    spec = ArchSpec.aggregating(4, 2, 2)
    assert spec.chunks == [(0, 5), (5, 5), (10, 5), (15, 5)]
    s2 = ArchSpec.aggregating(3, 2, 2)  # P=16, cs=5, leftover 1 -> last chunk 6
    assert s2.chunks[-1] == (10, 6)
    # P=14, chunk size 14//6=2 -> 7 chunks != 6 aggregates: the reference would crash (S4)
    with pytest.raises(ValueError):
        ArchSpec.aggregating(6, 1, 3)


def test_flatten_roundtrip():
    for spec in (ArchSpec.weightwise(3, 2), ArchSpec.recurrent(2, 3), ArchSpec.aggregating(4, 2, 2)):
        flat = np.arange(spec.P, dtype=np.float32)
        ws = spec.unflatten(flat)
        assert [w.shape for w in ws] == [tuple(s) for s in spec.layer_shapes]
        assert np.array_equal(spec.flatten(ws), flat)


def test_only_linear_supported():
    with pytest.raises(NotImplementedError):
        ArchSpec("weightwise", 2, 2, activation="sigmoid")


@pytest.mark.parametrize("w,d", [(2, 2), (8, 2), (16, 2), (32, 2), (8, 3), (16, 3), (12, 3), (5, 4)])
def test_recurrent_closed_form_tables(w, d):
    """csrc/srnn_generic.hip struct RD (the specialised Recurrent wave kernels) derives the
    SimpleRNN tables from (width, depth) alone: kernel of layer L at W + W^2 + (L-1) 2W^2
    (0 for L = 0), its recurrent kernel right after it, P = koff(D) + W + 1."""
    spec = ArchSpec.recurrent(w, d)
    offs, shapes = spec.offsets, spec.layer_shapes
    for L in range(d + 1):
        koff = 0 if L == 0 else w + w * w + (L - 1) * 2 * w * w
        i_n, u_n = (1 if L == 0 else w), (1 if L == d else w)
        assert offs[2 * L] == koff and shapes[2 * L] == (i_n, u_n)
        assert offs[2 * L + 1] == koff + i_n * u_n and shapes[2 * L + 1] == (u_n, u_n)
    koff_d = w + w * w + (d - 1) * 2 * w * w
    assert spec.P == koff_d + w + 1
