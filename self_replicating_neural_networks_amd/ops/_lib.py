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
ABI_VERSION = 14

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
OP_SCAN = 10
OP_RESPAWN = 11
OP_VARY_RUN = 12
OP_SOUP_PACK = 13
OP_SOUP_UNPACK = 14
OP_UID_ASSIGN = 15
OP_SOUP_GEN = 16
OP_GEN_FINISH = 17
OP_SOUP_PERMS = 18
OP_SOUP_SEQ = 19  # host: sequential (Gauss-Seidel) soup generations

FLAG_SHUFFLE = 1
FLAG_REMOVE_DIVERGENT = 2
FLAG_REMOVE_ZERO = 4
FLAG_FIX_SEC = 8
FLAG_ROW_FLAGS = 16
FLAG_RESPAWN_INLINE = 32
FLAG_COUNT_RESPAWNS = 64
FLAG_FULL_TABLE = 128
FLAG_STATS_X = 256
FLAG_GEN_ADVANCE = 512
FLAG_FUSED_CENSUS = 1024
FLAG_TWO_PHASE = 2048
FLAG_SHARDED_DECIDE = 4096
FLAG_MASKS_BS = 8192
FLAG_POST_UNPACK = 16384
FLAG_FINISH_PACK = 32768
FLAG_ASYNC_FINISH = 65536
FLAG_PRE_PERMS = 131072
FLAG_FINISH_BATCH = 262144
FLAG_GEN_POST = 524288   # sharded: uids + received-row index folded into the generation launch
FLAG_BORN_TOTAL = 1048576  # batched finish: each generation keeps its newborn count after its block stats
HELPER_CTL = 1 + 8192  # helper work-queue head + per-SIMD generation-wave counts (csrc/srnn_kernels.h)


class SrnnCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("kind", "width", "depth", "aggregates", "aggregator", "shuffler", "pp", "p", "dtype")]


_P = ctypes.c_void_p


class SrnnArgs(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int64), ("n_total", ctypes.c_int64), ("lo", ctypes.c_int64),
        ("steps", ctypes.c_int32), ("epochs", ctypes.c_int32), ("severity", ctypes.c_int32),
        ("early_exit", ctypes.c_int32), ("flags", ctypes.c_int32), ("gen", ctypes.c_int32),
        ("eps", ctypes.c_float), ("lr", ctypes.c_float),
        ("attacking_rate", ctypes.c_float), ("learn_from_rate", ctypes.c_float),
        ("seed", ctypes.c_uint64), ("ctr", ctypes.c_uint32), ("pad0", ctypes.c_uint32),
        ("W", _P), ("W2", _P), ("traj", _P),
        ("idx_f", _P), ("idx_t", _P), ("idx_o", _P), ("uid", _P),
        ("cls", _P), ("nsteps", _P), ("loss", _P), ("counts", _P),
        ("i32a", _P), ("i32b", _P), ("i32c", _P), ("i32d", _P), ("i32e", _P), ("i32f", _P),
        ("uid_out", _P), ("uid_base", _P), ("gen_ptr", _P), ("segment", ctypes.c_int64),
        ("world", ctypes.c_int32), ("rank", ctypes.c_int32), ("cap", ctypes.c_int64),
        ("sendbuf", _P), ("recvbuf", _P), ("need", _P), ("sendcnt", _P), ("rmap", _P), ("ovf", _P),
        ("stats", _P), ("census", _P),
        ("action", _P), ("counterpart", _P), ("respawn", _P),
        ("temp", _P), ("temp_bytes", ctypes.c_int64),
        ("dev", ctypes.c_int32), ("pad1", ctypes.c_int32), ("stream", _P), ("gen_out", _P),
        ("scratch", _P), ("scratch_bytes", ctypes.c_int64),
        ("perm_cur", _P), ("perm_next", _P), ("helper_ctl", _P), ("perm_e", ctypes.c_int32),
        ("helpers", ctypes.c_int32), ("temp2", _P), ("xdone", _P),
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
        L.srnn_scan_temp_bytes.argtypes = [ctypes.c_int64]
        L.srnn_scan_temp_bytes.restype = ctypes.c_int64
        L.srnn_is_generic.argtypes = [ctypes.POINTER(SrnnCfg), ctypes.c_int]
        L.srnn_is_generic.restype = ctypes.c_int
        L.srnn_generic_scratch_bytes.argtypes = [ctypes.POINTER(SrnnCfg), ctypes.c_int64, ctypes.c_int64]
        L.srnn_generic_scratch_bytes.restype = ctypes.c_int64
        L.srnn_set_force_generic.argtypes = [ctypes.c_int]
        L.srnn_set_force_generic.restype = None
        L.srnn_set_rnn_wave.argtypes = [ctypes.c_int]
        L.srnn_set_rnn_wave.restype = None
        vp, i64, cp = ctypes.c_void_p, ctypes.c_int64, ctypes.c_char_p
        for name, args in (("srnn_comm_available", [cp]), ("srnn_comm_unique_id", [cp, vp, ctypes.c_int]),
                           ("srnn_comm_init", [cp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_void_p)]),
                           ("srnn_comm_destroy", [vp, ctypes.c_int]), ("srnn_comm_async_error", [vp]),
                           ("srnn_comm_all_to_all", [vp, vp, vp, i64, vp]),
                           ("srnn_comm_all_gather", [vp, vp, vp, i64, vp]),
                           ("srnn_comm_all_reduce_i64", [vp, vp, vp, i64, vp])):
            f = getattr(L, name)
            f.argtypes = args
            f.restype = ctypes.c_int
        L.srnn_comm_library.restype = ctypes.c_char_p
        L.srnn_storage_encode.argtypes = [vp, vp, i64, ctypes.c_int, vp]
        L.srnn_storage_encode.restype = ctypes.c_int
        v = L.srnn_abi_version()
        if v != ABI_VERSION:
            raise NativeLibraryError(f"libsrnn ABI {v} != expected {ABI_VERSION}: rebuild with `make -C csrc`")
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


def set_force_generic(on: bool) -> None:
    """Route every op to the runtime-shape engine (A/B tests against the templated kernels)."""
    lib().srnn_set_force_generic(1 if on else 0)


def set_rnn_wave(on: bool) -> None:
    """Wide Recurrent nets wave per particle (default) or lane per particle (A/B tests)."""
    lib().srnn_set_rnn_wave(1 if on else 0)


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


def scan_temp_bytes(n: int) -> int:
    return int(lib().srnn_scan_temp_bytes(int(n)))


def last_error() -> str:
    return lib().srnn_last_error().decode(errors="replace")
