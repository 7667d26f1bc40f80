"""Process-global random streams of the compat API.

The reference never seeds anything: Keras initialisers, ``random.random()``
soup decisions and ``random.shuffle`` are all unseeded.  Here every random quantity is
a Philox stream keyed by a global seed, so runs are reproducible with ``set_seed`` and
still differ run-to-run by default (the seed is drawn from the OS at import).
"""
from __future__ import annotations

import itertools
import os
import random
import threading

_lock = threading.Lock()
_seed = int.from_bytes(os.urandom(8), "little") & 0xFFFFFFFFFFFF
_init_keys = itertools.count(1 << 40)
_op_ctr = itertools.count(1)
_py = random.Random(_seed)


def set_seed(seed: int) -> None:
    """Seed every stream of the compat API (inits, shuffles, soup decisions, vary)."""
    global _seed, _init_keys, _op_ctr, _py
    with _lock:
        _seed = int(seed)
        _init_keys = itertools.count(1 << 40)
        _op_ctr = itertools.count(1)
        _py = random.Random(_seed)


def get_seed() -> int:
    return _seed


def next_init_key() -> int:
    with _lock:
        return next(_init_keys)


def next_op() -> int:
    with _lock:
        return next(_op_ctr) & 0x3FFFFFF


def prng() -> float:
    """Uniform [0, 1) for sequential decisions (reference soup.prng, code/soup.py:6-7)."""
    with _lock:
        return _py.random()


def py_random() -> random.Random:
    return _py
