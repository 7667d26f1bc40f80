"""ctypes binding of ``libsrnn.so`` (csrc/): the native population kernels.

The library is built in-tree by ``csrc/Makefile`` (``hipcc --offload-arch=gfx950``) and
loaded with ``ctypes`` — no torch C++ extension machinery, so the .so has no libtorch
dependency and device pointers / the HIP stream are passed as plain integers
(``tensor.data_ptr()``, ``torch.cuda.current_stream().cuda_stream``).  Kernels launched
this way are captured by ``torch.cuda.CUDAGraph`` (a hipGraph on ROCm) like any other
launch on the capturing stream.

Field order of ``SrnnCfg``/``SrnnArgs`` mirrors ``csrc/srnn_abi.h``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# SRNN_LIB: load another build of the library (A/B of compiler flags on the GPU box)
LIB_PATH = os.environ.get("SRNN_LIB") or os.path.join(_HERE, "libsrnn.so")
CSRC = os.path.normpath(os.path.join(_HERE, "..", "..", "csrc"))
ABI_VERSION = 31

# SrnnOp (csrc/srnn_abi.h)
OP_INIT = 0
OP_APPLY = 1
OP_RUN_FIXPOINT = 2
OP_TRAIN = 3
OP_LEARN = 4
OP_CLASSIFY = 5
OP_PERTURB = 6
OP_SOUP_DECIDE = 7
OP_RESPAWN_SEQ = 8
OP_SOUP_EVOLVE = 9
OP_RESPAWN = 11
OP_VARY_RUN = 12
OP_UID_ASSIGN = 15
OP_SOUP_GEN = 16
OP_GEN_FINISH = 17
OP_SOUP_SEQ = 19  # sequential (Gauss-Seidel) soup generations
OP_X2_PACK = 20   # sharded soup, all-to-all exchange: finish + next decisions + rows (csrc/srnn_shard.hip)
OP_X2_POST = 21   # sharded soup: uids, census, received notices / requests
OP_SOUP_ORDERED = 22  # reference-order (sequential) generation, DAG-scheduled (csrc/srnn_ordered.h)
OP_SOUP_ORDERED_SH = 23  # one phase of a sharded reference-order generation (csrc/srnn_ordered_sh.h)
OP_ORD_PLAN = 24  # the plan of a reference-order generation (lists, versions, records, permutations)
OP_ORD_CENSUS = 25  # the census of a reference-order generation's final rows into its block stats
ORDSH_PLAN, ORDSH_LEVEL, ORDSH_PACK, ORDSH_UNPACK, ORDSH_CLOSE, ORDSH_LINK = range(6)
ORD_CTL_WORDS = 166   # o_ctl words of an ordered generation (csrc/srnn_ordered.h)
ORD_MAXLW, ORD_ERRW = 17, 18
ORD_BARW = 165        # phase-barrier arrivals of the in-run planning workgroups
ORD_NPART = 64        # partitions of the pending records
ORD_REC = 32          # int32 words per pending record
ORD_MAX_LEVELS = 16   # dependency levels reported one by one (deeper: one bin)


def ord_src_words(n: int) -> int:
    """int32 words of an n-turn ordered generation's o_src: [n][4] codes + level, [n] stored flags,
    [n] consumer-list heads, the pending records, the critical list, the ready queue."""
    n = max(int(n), 1)
    return 6 * n + (ORD_REC + 2) * ord_rec_total(n)


def ord_rec_total(n: int) -> int:
    """Pending-record capacity of an n-turn ordered generation (ord::rec_total: NPART partitions
    of ceil(ceil(n / 64) / NPART) * 64 records)."""
    return ORD_NPART * ((-(-n // 64) + ORD_NPART - 1) // ORD_NPART) * 64

# SrnnFlag bits (csrc/srnn_abi.h: one meaning each)
FLAG_SHUFFLE = 1 << 0
FLAG_REMOVE_DIVERGENT = 1 << 1
FLAG_REMOVE_ZERO = 1 << 2
FLAG_FIX_SEC = 1 << 3
FLAG_ROW_FLAGS = 1 << 4
FLAG_RESPAWN_INLINE = 1 << 5
FLAG_COUNT_RESPAWNS = 1 << 6
FLAG_FULL_TABLE = 1 << 7
FLAG_X2_PRIME = 1 << 8
FLAG_GEN_ADVANCE = 1 << 9
FLAG_FUSED_CENSUS = 1 << 10
FLAG_TWO_PHASE = 1 << 11
FLAG_MASKS_BS = 1 << 12
FLAG_GEN_COUNTS = 1 << 13
FLAG_FINISH_BATCH = 1 << 14
FLAG_BORN_TOTAL = 1 << 15
FLAG_X2 = 1 << 16
FLAG_X2_REMOTE = 1 << 17
FLAG_X2_FINISH_ONLY = 1 << 18
FLAG_X2_PRIO = 1 << 19
FLAG_X2_BOTH = 1 << 20
FLAG_X2_POST_FUSED = 1 << 21
FLAG_PTAB_READY = 1 << 23  # ptab already holds the generation's permutations (the sharded pack built them)
FLAG_ORD_PLANNED = 1 << 25  # OP_SOUP_ORDERED: the plan is already built (OP_ORD_PLAN one generation ahead)
FLAG_ORD_NEXT = 1 << 26  # OP_ORD_PLAN: plan generation gen + 1 (the one after the generation in flight)
FLAG_ORD_SYNC = 1 << 27  # OP_ORD_PLAN / OP_SOUP_ORDERED: ordered by the o_sync counters (two graphs, two streams)
FLAG_ORD_INPLAN = 1 << 28  # OP_SOUP_ORDERED: the run launch builds the next generation's plan (*_next buffers)
FLAG_ORD_CENSUS_LATER = 1 << 29  # OP_SOUP_ORDERED: the census is OP_ORD_CENSUS's, beside the next generation

X2_HDR = 12           # int64 header words of an exchange block
X2_REMOTE_WAVES = 4096
NIL = 0xFFFFFFFF      # end of an attack list


class SrnnCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("kind", "width", "depth", "aggregates", "aggregator", "shuffler", "pp", "p", "dtype")]


_P = ctypes.c_void_p
_I64, _I32 = ctypes.c_int64, ctypes.c_int32


class SrnnArgs(ctypes.Structure):
    _fields_ = [
        ("n", _I64), ("n_total", _I64), ("lo", _I64),
        ("steps", _I32), ("epochs", _I32), ("severity", _I32),
        ("early_exit", _I32), ("flags", ctypes.c_uint32), ("gen", _I32),
        ("eps", ctypes.c_float), ("lr", ctypes.c_float),
        ("attacking_rate", ctypes.c_float), ("learn_from_rate", ctypes.c_float),
        ("seed", ctypes.c_uint64), ("ctr", ctypes.c_uint32), ("x_emul", ctypes.c_uint32),
        ("W", _P), ("W2", _P), ("traj", _P),
        ("idx_f", _P), ("idx_t", _P), ("idx_o", _P), ("uid", _P),
        ("cls", _P), ("nsteps", _P), ("loss", _P), ("counts", _P),
        # soup: decisions and attack lists
        ("heads", _P), ("nexts", _P), ("heads_next", _P), ("nexts_next", _P),
        ("dec_at", _P), ("dec_te", _P), ("ballots", _P), ("rowflags", _P), ("done", _P),
        ("uid_out", _P), ("uid_base", _P), ("gen_ptr", _P), ("gen_out", _P), ("segment", _I64),
        ("world", _I32), ("rank", _I32),
        # sharded exchange
        ("x_cr", _I64), ("x_cn", _I64), ("x_cq", _I64), ("x_blk", _I64),
        ("sendbuf", _P), ("recvbuf", _P), ("stats", _P), ("census", _P), ("err", _P),
        ("x_dep", _P), ("x_dep_next", _P), ("x_rlist", _P), ("x_rlist_next", _P),
        ("x_rcount", _P), ("x_rcount_next", _P), ("x_rslot", _P), ("x_rslot_next", _P),
        ("x_satt", _P), ("x_satt_next", _P), ("x_cno", _P), ("x_cno_next", _P),
        ("x_crq", _P), ("x_crq_next", _P), ("x_srep", _P), ("x_nsrep", _P),
        ("x_part", _P), ("x_ctl", _P), ("x_groups", _I32), ("pad2", _I32), ("x_hpre", _P), ("x_hgrp", _P), ("temp2", _P),
        ("action", _P), ("counterpart", _P), ("respawn", _P),
        ("temp", _P), ("temp_bytes", _I64),
        ("dev", _I32), ("pad1", _I32), ("stream", _P),
        ("scratch", _P), ("scratch_bytes", _I64),
        # ordered (reference-order) generation
        ("W3", _P), ("o_src", _P), ("o_list", _P), ("o_ctl", _P), ("o_levels", _I32), ("pad3", _I32),
        # precomputed SGD epoch permutations of a soup generation
        ("ptab", _P),
        # ordered generation trace (debug): [n][2] start / end times of each turn (100 MHz)
        ("o_trace", _P),
        # the sharded reference-order generation: this rank's turns [o_lo, o_hi)
        ("o_lo", _I64), ("o_hi", _I64),
        # SRNN_F_ORD_INPLAN: the next generation's plan set, built by the run launch's last workgroups
        ("o_src_next", _P), ("o_list_next", _P), ("o_ctl_next", _P), ("ptab_next", _P),
        ("o_plan_groups", _I32), ("o_bulk_delay", _I32), ("o_sync", _P), ("o_shadow", _I32), ("pad5", _I32), ("o_census_temp", _P),
    ]


class NativeLibraryError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()


def build(force: bool = False, jobs: int = 8) -> str:
    """Compile libsrnn.so for gfx950 in-tree (make -C csrc)."""
    cmd = ["make", "-C", CSRC, f"-j{jobs}"]
    if force:
        subprocess.run(["make", "-C", CSRC, "clean"], check=True)
    subprocess.run(cmd, check=True)
    return LIB_PATH


def lib():
    """Load libsrnn.so; raise loudly if it is missing (no silent eager fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            if os.environ.get("SRNN_AUTOBUILD", "1") == "1" and os.path.isdir(CSRC):
                build()
            else:
                raise NativeLibraryError(f"{LIB_PATH} is missing: run `make -C csrc` (hipcc, gfx950)")
        L = ctypes.CDLL(LIB_PATH)
        L.srnn_abi_version.restype = ctypes.c_int
        L.srnn_has_config.argtypes = [ctypes.POINTER(SrnnCfg)]
        L.srnn_has_config.restype = ctypes.c_int
        L.srnn_run.argtypes = [ctypes.c_int, ctypes.POINTER(SrnnCfg), ctypes.POINTER(SrnnArgs)]
        L.srnn_run.restype = ctypes.c_int
        L.srnn_last_error.restype = ctypes.c_char_p
        L.srnn_is_generic.argtypes = [ctypes.POINTER(SrnnCfg), ctypes.c_int]
        L.srnn_is_generic.restype = ctypes.c_int
        L.srnn_supports.argtypes = [ctypes.POINTER(SrnnCfg), ctypes.c_int, ctypes.c_int]
        L.srnn_supports.restype = ctypes.c_int
        L.srnn_generic_scratch_bytes.argtypes = [ctypes.POINTER(SrnnCfg), ctypes.c_int64, ctypes.c_int64]
        L.srnn_generic_scratch_bytes.restype = ctypes.c_int64
        L.srnn_set_force_generic.argtypes = [ctypes.c_int]
        L.srnn_set_force_generic.restype = None
        L.srnn_set_rnn_wave.argtypes = [ctypes.c_int]
        L.srnn_set_rnn_wave.restype = None
        L.srnn_set_ww_wave.argtypes = [ctypes.c_int]
        L.srnn_set_ww_wave.restype = None
        L.srnn_set_rnn_spec.argtypes = [ctypes.c_int]
        L.srnn_set_rnn_spec.restype = None
        L.srnn_set_rnn_soup.argtypes = [ctypes.c_int]
        L.srnn_set_rnn_soup.restype = None
        vp, i64, cp = ctypes.c_void_p, ctypes.c_int64, ctypes.c_char_p
        for name, args in (("srnn_comm_available", [cp]), ("srnn_comm_unique_id", [cp, vp, ctypes.c_int]),
                           ("srnn_comm_init", [cp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_void_p)]),
                           ("srnn_comm_destroy", [vp, ctypes.c_int]), ("srnn_comm_async_error", [vp]),
                           ("srnn_comm_all_to_all", [vp, vp, vp, i64, vp]),
                           ("srnn_comm_all_gather", [vp, vp, vp, i64, vp]),
                           ("srnn_comm_all_reduce_i64", [vp, vp, vp, i64, vp]),
                           ("srnn_comm_count", [vp]), ("srnn_comm_user_rank", [vp]),
                           ("srnn_set_knob", [ctypes.c_int, ctypes.c_int]), ("srnn_get_knob", [ctypes.c_int]),
                           ("srnn_stream_probe", [vp, vp, vp, i64])):
            f = getattr(L, name)
            f.argtypes = args
            f.restype = ctypes.c_int
        L.srnn_set_knob.restype = None
        L.srnn_comm_library.restype = ctypes.c_char_p
        L.srnn_storage_encode.argtypes = [vp, vp, i64, ctypes.c_int, vp]
        L.srnn_storage_encode.restype = ctypes.c_int
        v = L.srnn_abi_version()
        if v != ABI_VERSION:
            raise NativeLibraryError(f"libsrnn ABI {v} != expected {ABI_VERSION}: rebuild with `make -C csrc`")
        L.srnn_args_size.restype = ctypes.c_int64
        L.srnn_cfg_size.restype = ctypes.c_int64
        if (L.srnn_args_size(), L.srnn_cfg_size()) != (ctypes.sizeof(SrnnArgs), ctypes.sizeof(SrnnCfg)):
            raise NativeLibraryError(f"SrnnArgs/SrnnCfg layout mismatch: library {L.srnn_args_size()}/"
                                     f"{L.srnn_cfg_size()} bytes, ctypes {ctypes.sizeof(SrnnArgs)}/"
                                     f"{ctypes.sizeof(SrnnCfg)}")
        _lib = L
        return _lib


DTYPE_FP32, DTYPE_BF16, DTYPE_FP16 = 0, 1, 2


def make_cfg(spec, dtype: int = DTYPE_FP32) -> SrnnCfg:
    return SrnnCfg(*spec.native_cfg_tuple(), int(dtype))


def has_config(spec, dtype: int = DTYPE_FP32) -> bool:
    return bool(lib().srnn_has_config(ctypes.byref(make_cfg(spec, dtype))))


def is_generic(spec, op: int, dtype: int = DTYPE_FP32) -> bool:
    """True when ``op`` of this architecture runs on the runtime-shape engine
    (csrc/srnn_generic.hip) on the GPU instead of a shape-specialised kernel."""
    return bool(lib().srnn_is_generic(ctypes.byref(make_cfg(spec, dtype)), int(op)))


def supports(spec, op: int, device: bool, dtype: int = DTYPE_FP32) -> bool:
    """True when ``op`` of this architecture has a native implementation on the device
    (``device=True``) or on the host."""
    return bool(lib().srnn_supports(ctypes.byref(make_cfg(spec, dtype)), int(op), 1 if device else 0))


# execution knobs (csrc/srnn_abi.h SrnnKnob; config.py ExecConfig): the environment variable
# of a knob, when set, overrides what is set here
KNOBS = {"force_generic": 0, "rnn_wave": 1, "rnn_spec": 2, "rnn_soup": 3, "ww_wave": 4, "big_wave": 5,
         "fix_group": 6, "soup_lanes": 7, "ord_crit": 8, "ord_queue": 9, "ord_shadow": 10, "ord_bulk_delay": 11}
KNOB_ENV = {"force_generic": "SRNN_FORCE_GENERIC", "rnn_wave": "SRNN_RNN_WAVE", "rnn_spec": "SRNN_RNN_SPEC",
            "rnn_soup": "SRNN_RNN_SOUP", "ww_wave": "SRNN_WW_WAVE", "big_wave": "SRNN_BIG_WAVE",
            "fix_group": "SRNN_FIX_GROUP", "soup_lanes": "SRNN_SOUP_LANES", "ord_crit": "SRNN_ORD_CRIT",
            "ord_queue": "SRNN_ORD_QUEUE", "ord_shadow": "SRNN_ORD_SHADOW", "ord_bulk_delay": "SRNN_ORD_BULK_DELAY"}


def streams_concurrent(side, main, device, timeout_us: int = 20000) -> bool:
    """True when kernels on the two torch streams run at the same time (a waiter on ``side`` sees
    the flag a setter on ``main`` raises within ``timeout_us``): False under a profiler that
    serialises kernels or when the two streams share one hardware queue."""
    import torch
    flag = torch.zeros(2, dtype=torch.int32, device=device)
    torch.cuda.synchronize(device)
    if lib().srnn_stream_probe(ctypes.c_void_p(flag.data_ptr()), ctypes.c_void_p(side.cuda_stream),
                               ctypes.c_void_p(main.cuda_stream), int(timeout_us)) != 0:
        return False
    torch.cuda.synchronize(device)
    return int(flag[1].item()) == 1


def set_knob(name: str, value: int) -> None:
    """Set a library execution knob (-1: back to the built-in default)."""
    lib().srnn_set_knob(KNOBS[name], int(value))


def get_knob(name: str) -> int:
    """The knob's value in force (environment override included); -1 = built-in default."""
    return int(lib().srnn_get_knob(KNOBS[name]))


def set_force_generic(on: bool) -> None:
    """Route every op to the runtime-shape engine (A/B tests against the templated kernels)."""
    lib().srnn_set_force_generic(1 if on else 0)


def set_rnn_wave(on: bool) -> None:
    """Wide Recurrent nets wave per particle (default) or lane per particle (A/B tests)."""
    lib().srnn_set_rnn_wave(1 if on else 0)


def set_rnn_spec(on: bool) -> None:
    """Width / depth-specialised Recurrent wave kernels for RNN(8|16|32, 2) and RNN(8|16, 3) (default) or the
    runtime-shape wave kernel for every width (A/B tests)."""
    lib().srnn_set_rnn_spec(1 if on else 0)


def set_rnn_soup(on: bool) -> None:
    """Single-rank soup generations of wide Recurrent nets wave per particle (default) or on the
    lane path (A/B tests)."""
    lib().srnn_set_rnn_soup(1 if on else 0)


def set_ww_wave(on: bool) -> None:
    """Runtime-shape Weightwise training on lanes-per-particle waves (default) or lane per
    particle (A/B tests)."""
    lib().srnn_set_ww_wave(1 if on else 0)


def generic_scratch_bytes(spec, n: int, dtype: int = DTYPE_FP32, max_lanes: int = 65536) -> int:
    """Device scratch the runtime-shape engine needs for ``n`` rows (per-lane vectors)."""
    return int(lib().srnn_generic_scratch_bytes(ctypes.byref(make_cfg(spec, dtype)), int(n), int(max_lanes)))


def run(op: int, spec, args: SrnnArgs, cfg: SrnnCfg = None, dtype: int = DTYPE_FP32) -> None:
    L = lib()
    cfg = cfg if cfg is not None else make_cfg(spec, dtype)
    r = L.srnn_run(op, ctypes.byref(cfg), ctypes.byref(args))
    if r != 0:
        msg = L.srnn_last_error().decode(errors="replace")
        raise NativeLibraryError(f"srnn op {op} failed ({r}): {msg} [spec={spec}]")


def last_error() -> str:
    return lib().srnn_last_error().decode(errors="replace")
