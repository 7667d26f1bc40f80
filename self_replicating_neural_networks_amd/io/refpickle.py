"""Reference-schema pickles: writer and restricted (code-free) reader.

The reference persists experiments with ``dill`` (protocol 3): ``experiment.dill`` /
``trajectorys.dill`` hold an ``experiment.Experiment`` instance, ``soup.dill`` a
``soup.Soup`` instance (particles replaced by ``{uid: [state dicts]}``), ``all_*.dill``
plain lists.  Its ``Soup.generator`` is a dill-pickled *Python 3.6 code
object* — untrusted and not rebuildable.

* ``dump`` writes the same schema: our objects are emitted under the global names
  ``experiment Experiment`` / ``soup Soup``; tensors become numpy arrays; the soup
  generator becomes a plain dict describing the architecture (data, not code).
* ``load`` uses an ``Unpickler`` whose ``find_class`` admits only numpy reconstruction
  helpers and maps every other global to an inert record or stub: no function or code
  object from the file is ever called or built.
"""
from __future__ import annotations

import copyreg
import io
import pickle
from typing import Any

import numpy as np

PROTOCOL = 3


class RefRecord:
    """Attribute bag standing for a pickled reference object."""

    _ref_global = ("builtins", "object")

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def __setstate__(self, state):
        if isinstance(state, tuple) and len(state) == 2:  # (dict, slots)
            state = {**(state[0] or {}), **(state[1] or {})}
        if isinstance(state, dict):
            self.__dict__.update(state)
        else:
            self.__dict__["_state"] = state

    def __repr__(self):
        keys = ", ".join(sorted(self.__dict__)[:8])
        return f"<{self._ref_global[0]}.{self._ref_global[1]} record: {keys}>"


class ExperimentRecord(RefRecord):
    _ref_global = ("experiment", "Experiment")


class SoupRecord(RefRecord):
    _ref_global = ("soup", "Soup")


_RECORD_CLASSES = {("experiment", "Experiment"): ExperimentRecord, ("soup", "Soup"): SoupRecord}


class Opaque:
    """Inert placeholder for a global the reader refuses to import (functions, code, ...)."""

    def __init__(self, module, name, args=()):
        self.module, self.name, self.args = module, name, args

    def __repr__(self):
        return f"<opaque {self.module}.{self.name}>"

    def __call__(self, *args, **kwargs):  # e.g. a stubbed type being "instantiated": stays inert
        return Opaque(self.module, self.name)

    def __setstate__(self, state):
        self.state = state


def _opaque_factory(module, name):
    def make(*args, **kwargs):
        return Opaque(module, name, ())  # arguments (e.g. code bytes) are dropped, never used
    make.__name__ = f"opaque_{name}"
    return make


def _generic_record(module, name):
    return type(name, (RefRecord,), {"_ref_global": (module, name)})


# ------------------------------------------------------------------------------ reader
class RestrictedUnpickler(pickle.Unpickler):
    _NUMPY = {
        ("numpy", "ndarray"): np.ndarray,
        ("numpy", "dtype"): np.dtype,
    }

    def find_class(self, module, name):
        if (module, name) in self._NUMPY:
            return self._NUMPY[(module, name)]
        if module in ("numpy.core.multiarray", "numpy._core.multiarray") and name in ("_reconstruct", "scalar"):
            from numpy.core import multiarray as ma  # noqa: deprecated alias kept by numpy 2
            return getattr(ma, name)
        if module == "numpy" and name in ("float32", "float64", "int64", "int32", "bool_"):
            return getattr(np, name)
        if (module, name) in _RECORD_CLASSES:
            return _RECORD_CLASSES[(module, name)]
        if module in ("experiment", "soup", "network", "util", "__main__") and name[:1].isupper():
            return _generic_record(module, name)
        if module == "builtins" and name in ("set", "frozenset", "list", "dict", "tuple", "complex"):
            return {"set": set, "frozenset": frozenset, "list": list, "dict": dict, "tuple": tuple,
                    "complex": complex}[name]
        if module == "copyreg" and name == "_reconstructor":
            return _safe_reconstructor
        if module == "dill._dill" and name == "_import_module":
            return _ModuleRef
        if module == "dill._dill" and name == "_get_attr":
            return _safe_get_attr
        # dill function / code / type / module helpers and anything else: inert stubs
        return _opaque_factory(module, name)


_NUMPY_FUNCS = {("numpy.core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "scalar"),
                ("numpy.core._multiarray_umath", "_reconstruct"), ("numpy.core._multiarray_umath", "scalar"),
                ("numpy._core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "scalar")}


class _ModuleRef:
    """dill `_import_module(name)`: remembers the name, imports nothing."""

    def __init__(self, name, *args, **kwargs):
        self.name = name


def _safe_get_attr(obj, name):
    """dill `_get_attr(module, name)`: resolves only allow-listed numpy reconstruction helpers
    (older dill writes numpy arrays this way); anything else stays inert."""
    if isinstance(obj, _ModuleRef) and (obj.name, name) in _NUMPY_FUNCS:
        from numpy.core import multiarray as ma  # noqa
        return getattr(ma, name)
    return Opaque(getattr(obj, "name", "?"), name)


def _safe_reconstructor(cls, base, state):
    if isinstance(cls, type) and issubclass(cls, RefRecord):
        obj = cls.__new__(cls)
        return obj
    return Opaque("copyreg", "_reconstructor")


def load(path_or_file) -> Any:
    if hasattr(path_or_file, "read"):
        return RestrictedUnpickler(path_or_file).load()
    with open(path_or_file, "rb") as f:
        return RestrictedUnpickler(f).load()


def loads(data: bytes) -> Any:
    return RestrictedUnpickler(io.BytesIO(data)).load()


# ------------------------------------------------------------------------------ writer
def _to_ref(obj, memo=None):
    """Convert framework objects into reference-schema data (records, numpy, builtins)."""
    import torch  # local: keep the reader importable without torch

    memo = {} if memo is None else memo
    oid = id(obj)
    if oid in memo:
        return memo[oid]
    if isinstance(obj, RefRecord):
        rec = obj.__class__.__new__(obj.__class__)
        memo[oid] = rec
        rec.__dict__.update({k: _to_ref(v, memo) for k, v in obj.__dict__.items()})
        return rec
    if torch.is_tensor(obj):
        return obj.detach().cpu().numpy()
    if isinstance(obj, (np.ndarray, np.generic, str, bytes, int, float, bool, type(None), complex)):
        return obj
    if isinstance(obj, dict):
        d = {}
        memo[oid] = d
        for k, v in obj.items():
            d[_to_ref(k, memo)] = _to_ref(v, memo)
        return d
    if isinstance(obj, list):
        lst = []
        memo[oid] = lst
        lst.extend(_to_ref(v, memo) for v in obj)
        return lst
    if isinstance(obj, tuple):
        return tuple(_to_ref(v, memo) for v in obj)
    if isinstance(obj, (set, frozenset)):
        return type(obj)(_to_ref(v, memo) for v in obj)
    to_ref = getattr(obj, "__ref_record__", None)
    if to_ref is not None:
        rec = to_ref()
        memo[oid] = rec
        return _to_ref(rec, memo)
    # our Experiment classes map to experiment.Experiment (reference __copy__ downgrades too)
    from ..experiment import Experiment
    if isinstance(obj, Experiment):
        state = obj.__getstate__() if hasattr(obj, "__getstate__") else dict(obj.__dict__)
        rec = ExperimentRecord.__new__(ExperimentRecord)
        memo[oid] = rec
        rec.__dict__.update({k: _to_ref(v, memo) for k, v in state.items()})
        return rec
    from ..arch import ArchSpec
    if isinstance(obj, ArchSpec):
        import dataclasses
        return dataclasses.asdict(obj)
    # network facades / anything else with weights: store its flat weights
    gw = getattr(obj, "get_weights", None)
    if callable(gw):
        try:
            return [np.asarray(w) for w in gw()]
        except Exception:  # pragma: no cover
            pass
    return repr(obj)


class _RefPickler(pickle._Pickler):
    def save_global(self, obj, name=None):
        ref = obj.__dict__.get("_ref_global") if isinstance(obj, type) and issubclass(obj, RefRecord) else None
        if ref is None and isinstance(obj, type) and issubclass(obj, RefRecord):
            ref = obj._ref_global
        if ref is not None:
            self.write(pickle.GLOBAL + f"{ref[0]}\n{ref[1]}\n".encode("utf-8"))
            self.memoize(obj)
            return
        return super().save_global(obj, name)

    def reducer_override(self, obj):
        if isinstance(obj, RefRecord):
            return (copyreg.__newobj__, (type(obj),), dict(obj.__dict__))
        return NotImplemented


def dumps(obj) -> bytes:
    buf = io.BytesIO()
    _RefPickler(buf, protocol=PROTOCOL).dump(_to_ref(obj))
    return buf.getvalue()


def dump(obj, path) -> None:
    with open(path, "wb") as f:
        f.write(dumps(obj))


def globals_of(data: bytes):
    """Set of (module, name) globals referenced by a pickle (for schema tests)."""
    import pickletools
    out = set()
    for op, arg, _ in pickletools.genops(data):
        if op.name == "GLOBAL":
            m, n = arg.split(" ", 1)
            out.add((m, n))
        elif op.name == "STACK_GLOBAL":
            out.add(("<stack>", "<stack>"))
    return out
