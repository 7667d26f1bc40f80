"""Tracing / profiling helpers (the reference has only tqdm bars).

* :func:`roctx_range` -- named ranges in the ROCm tracer timeline (``rocprofv3
  --marker-trace``).  The native library additionally opens one range per operator launch
  when ``SRNN_ROCTX=1`` (csrc/srnn_common.hip, resolved with ``dlopen`` so there is no link
  dependency).
* :class:`PhaseTimer` -- hipEvent timing of named phases on the current stream (no host
  synchronisation until :meth:`PhaseTimer.summary`).
* :func:`rocprof_commands` -- the profiling recipe for this pool as command lines: one
  ``--kernel-trace --stats`` run, then counter passes that respect the per-block counter
  limits of one ``--pmc`` run (never combined with a tracing domain).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from collections import defaultdict
from typing import Dict, List, Optional

_ROCTX = None
_ROCTX_TRIED = False
_LIBS = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so")


def _roctx():
    global _ROCTX, _ROCTX_TRIED
    if not _ROCTX_TRIED:
        _ROCTX_TRIED = True
        for name in _LIBS:
            for path in (name, os.path.join("/opt/rocm/lib", name)):
                try:
                    lib = ctypes.CDLL(path)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                    _ROCTX = lib
                    return _ROCTX
                except (OSError, AttributeError):
                    continue
    return _ROCTX


def roctx_available() -> bool:
    return _roctx() is not None


@contextlib.contextmanager
def roctx_range(name: str):
    """Push/pop a roctx range (no-op when the library is absent)."""
    lib = _roctx()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def roctx_mark(name: str):
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


class PhaseTimer:
    """Accumulates device time per named phase with hipEvents (torch.cuda.Event on ROCm).
    On CPU tensors it falls back to host wall time."""

    def __init__(self, device=None):
        import torch
        self.torch = torch
        self.device = torch.device(device) if device is not None else None
        self.cuda = self.device is not None and self.device.type == "cuda"
        self._pending: List = []
        self.totals: Dict[str, float] = defaultdict(float)
        self.calls: Dict[str, int] = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        if self.cuda:
            a = self.torch.cuda.Event(enable_timing=True)
            b = self.torch.cuda.Event(enable_timing=True)
            a.record()
            with roctx_range(name):
                yield
            b.record()
            self._pending.append((name, a, b))
        else:
            import time
            t0 = time.perf_counter()
            with roctx_range(name):
                yield
            self.totals[name] += (time.perf_counter() - t0) * 1e3
            self.calls[name] += 1

    def summary(self) -> Dict[str, Dict[str, float]]:
        """{phase: {"ms": total, "calls": n, "ms_per_call": avg}} (synchronises)."""
        if self._pending:
            self.torch.cuda.synchronize(self.device)
            for name, a, b in self._pending:
                self.totals[name] += a.elapsed_time(b)
                self.calls[name] += 1
            self._pending.clear()
        return {k: dict(ms=v, calls=self.calls[k], ms_per_call=v / max(self.calls[k], 1))
                for k, v in sorted(self.totals.items())}


# counters per hardware block that one --pmc pass may hold on gfx950 (pool rule)
PMC_BLOCK_LIMITS = {"SQ": 8, "TCC": 4, "TCP": 4, "TA": 2, "TD": 2, "GRBM": 2}
# counters that occupy more than one TCC slot
_TCC_COST = {"FETCH_SIZE": 3, "WRITE_SIZE": 2}

PMC_SETS = {
    "valu_mfma": ["SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES",
                  "SQ_WAVES", "SQ_INSTS_LDS", "GRBM_GUI_ACTIVE"],
    "lds": ["SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM",
            "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "SQ_INST_CYCLES_VALU"],
    "hbm": ["FETCH_SIZE", "GRBM_GUI_ACTIVE", "GRBM_COUNT"],
}


def _block(counter: str) -> str:
    if counter in _TCC_COST:
        return "TCC"
    return counter.split("_", 1)[0]


def check_pmc_pass(counters: List[str]) -> None:
    """Raise ValueError if one --pmc pass would exceed a block's counter limit (the run
    would hang after 'error code 38')."""
    use: Dict[str, int] = defaultdict(int)
    seen = set()
    for c in counters:
        base = c
        for suf in ("_sum", "_avr", "_min", "_max"):
            if base.endswith(suf):
                base = base[: -len(suf)]
        if base in seen:
            continue
        seen.add(base)
        blk = _block(base)
        use[blk] += _TCC_COST.get(base, 1)
    for blk, n in use.items():
        lim = PMC_BLOCK_LIMITS.get(blk)
        if lim is not None and n > lim:
            raise ValueError(f"--pmc pass uses {n} {blk} counters (limit {lim}): split it")


def rocprof_commands(cmd: List[str], out_dir: str = "gpurun_out/prof", sets: Optional[List[str]] = None,
                     timeout_s: int = 120) -> List[List[str]]:
    """Command lines of the profiling recipe: one kernel-trace/stats run and one run per
    counter set.  The program itself follows ``--`` (no env / shell hops)."""
    out = [["timeout", "-k", "10", str(timeout_s), "rocprofv3", "--kernel-trace", "--stats", "-d", out_dir,
            "-o", "trace", "--output-format", "csv", "--"] + list(cmd)]
    for s in sets or []:
        counters = PMC_SETS[s]
        check_pmc_pass(counters)
        out.append(["timeout", "-s", "KILL", "60", "rocprofv3", "--pmc"] + counters +
                   ["-d", f"{out_dir}_{s}", "-o", s, "--output-format", "csv", "--"] + list(cmd))
    return out
