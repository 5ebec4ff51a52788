"""ctypes binding of the C ABI in include/fcr.h (libfcr.so, built for gfx950).

The library is the only compute path of this package: if it is missing or fails to load, every
entry point raises — there is no CPU or eager-PyTorch fallback.
"""
from __future__ import annotations

import ctypes
import os
import sys
import threading

_LIB_NAME = "libfcr.so"
_HERE = os.path.dirname(os.path.abspath(__file__))
_IN_TREE = os.path.join(_HERE, "lib", _LIB_NAME)
# FCR_LIB: another build of the same ABI (A/B timing, scripts/inject_stale_lo.sh's fault-injected build). A development
# switch only: it takes effect together with FCR_DEV=1 (load() refuses FCR_LIB without it and says on stderr which
# library it loaded when it is honoured); the in-tree library otherwise.
LIB_PATH = os.environ.get("FCR_LIB") or _IN_TREE

FCR_OK = 0
# 6 (round 6): kept wide windows store gate activations (not pre-activations), fcr_wide_bwd_cell[_workspace] exported
ABI_VERSION = 6
PRECISION_FP32, PRECISION_F16 = 0, 1
ERRORS = {-1: "FCR_EINVAL", -2: "FCR_EWORKSPACE", -3: "FCR_EHIP", -4: "FCR_EUNSUPPORTED"}

# Every symbol include/fcr.h declares (tests check the .so exports exactly these).
EXPORTS = ("fcr_workspace_size", "fcr_wide_kept_windows", "fcr_forward", "fcr_backward", "fcr_lstm_workspace_size",
           "fcr_lstm_forward", "fcr_lstm_backward", "fcr_plant_rk4", "fcr_closed_loop_run", "fcr_window_gather",
           "fcr_fnn_workspace_size", "fcr_fnn_forward", "fcr_fnn_backward", "fcr_set_small_batch_limit",
           "fcr_get_small_batch_limit", "fcr_set_small_pipe_limit", "fcr_get_small_pipe_limit", "fcr_set_small_pipe_sets",
           "fcr_get_small_pipe_sets", "fcr_set_wide_keep_budget", "fcr_get_wide_keep_budget", "fcr_last_error",
           "fcr_abi_version", "fcr_wide_bwd_cell_workspace", "fcr_wide_bwd_cell")
OPT_INHERIT, KEEP_AUTO = -2, -1
INT32_MAX, INT64_MAX = 2**31 - 1, 2**63 - 1


class FcrDims(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int32), ("N", ctypes.c_int32), ("L", ctypes.c_int32), ("H", ctypes.c_int32),
        ("layers", ctypes.c_int32), ("in_dim", ctypes.c_int32), ("out_dim", ctypes.c_int32),
        ("ctrl_in", ctypes.c_int32), ("ctrl_hidden", ctypes.c_int32), ("alpha", ctypes.c_float),
        ("precision", ctypes.c_int32),
    ]


class FcrOptions(ctypes.Structure):
    """fcr_options (include/fcr.h): the per-call kernel options; `kernels` is written by each call."""
    _fields_ = [("small_batch_limit", ctypes.c_int32), ("kernels", ctypes.c_int32), ("wide_keep_budget", ctypes.c_int64)]


def make_options(small_batch_limit=None, wide_keep_budget=None) -> FcrOptions:
    """Per-call options: None inherits the process-wide default; wide_keep_budget "auto" = the library's policy."""
    keep = OPT_INHERIT if wide_keep_budget is None else KEEP_AUTO if wide_keep_budget == "auto" else int(wide_keep_budget)
    if wide_keep_budget is not None and not KEEP_AUTO <= keep <= INT64_MAX:
        raise ValueError(f"wide_keep_budget must be 0..2**63-1 bytes, 'auto' or None, got {wide_keep_budget!r}")
    small = OPT_INHERIT if small_batch_limit is None else int(small_batch_limit)
    # the fields are c_int32 / c_int64: a value outside them would wrap silently into INHERIT or 'never'
    if small_batch_limit is not None and not 0 <= small <= INT32_MAX:
        raise ValueError(f"small_batch_limit must be 0..2**31-1 or None, got {small_batch_limit!r}")
    return FcrOptions(small, 0, keep)


class FcrWeights(ctypes.Structure):
    _fields_ = [
        ("ctrl_w_inp", ctypes.c_void_p), ("ctrl_b_inp", ctypes.c_void_p), ("ctrl_w_out", ctypes.c_void_p),
        ("w_ih", ctypes.c_void_p * 3), ("w_hh", ctypes.c_void_p * 3),
        ("fc_w", ctypes.c_void_p), ("fc_b", ctypes.c_void_p),
    ]


class FcrWindows(ctypes.Structure):
    _fields_ = [
        ("rows", ctypes.c_int64), ("traj_len", ctypes.c_int32), ("lookback", ctypes.c_int32),
        ("nx", ctypes.c_int32), ("ny", ctypes.c_int32), ("nz", ctypes.c_int32),
        ("X", ctypes.c_void_p), ("Y", ctypes.c_void_p), ("Z", ctypes.c_void_p),
    ]


class FcrClosedLoop(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int32), ("T", ctypes.c_int32), ("ts", ctypes.c_double),
        ("substeps", ctypes.c_int32), ("smooth", ctypes.c_int32),
        ("x0", ctypes.c_void_p), ("ref", ctypes.c_void_p),
        ("ctrl_w_inp", ctypes.c_void_p), ("ctrl_b_inp", ctypes.c_void_p), ("ctrl_w_out", ctypes.c_void_p),
        ("ctrl_hidden", ctypes.c_int32), ("in_scale", ctypes.c_double * 2),
        ("ref_scale", ctypes.c_double), ("out_scale", ctypes.c_double),
        ("x", ctypes.c_void_p), ("u", ctypes.c_void_p),
    ]


class NativeError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()


def load() -> ctypes.CDLL:
    """Load libfcr.so once (raises NativeError with build instructions if absent)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if LIB_PATH != _IN_TREE:
            if os.environ.get("FCR_DEV") != "1":
                raise NativeError(f"FCR_LIB={LIB_PATH} names a development build; set FCR_DEV=1 to load it "
                                  "(unset FCR_LIB for the in-tree library)")
            sys.stderr.write(f"forging_control_amd: FCR_LIB development build {LIB_PATH}\n")
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(hipcc --offload-arch=gfx950). There is no fallback path.")
        lib = ctypes.CDLL(LIB_PATH)
        vp, i32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        po = ctypes.POINTER(FcrOptions)
        lib.fcr_workspace_size.argtypes = [ctypes.POINTER(FcrDims), po, i32, ctypes.POINTER(sz)]
        lib.fcr_workspace_size.restype = i32
        lib.fcr_wide_kept_windows.argtypes = [ctypes.POINTER(FcrDims), sz, ctypes.POINTER(ctypes.c_int32)]
        lib.fcr_wide_kept_windows.restype = i32
        lib.fcr_forward.argtypes = [ctypes.POINTER(FcrDims), po, ctypes.POINTER(FcrWeights),
                                    vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp, sz, vp]
        lib.fcr_forward.restype = i32
        lib.fcr_backward.argtypes = [ctypes.POINTER(FcrDims), po, vp, vp, vp, vp, vp, vp, vp, vp, vp, sz, vp]
        lib.fcr_backward.restype = i32
        lib.fcr_plant_rk4.argtypes = [i32, i32, ctypes.c_double, i32, i32, vp, vp, vp, vp]
        lib.fcr_plant_rk4.restype = i32
        lib.fcr_lstm_workspace_size.argtypes = [ctypes.POINTER(FcrDims), i32, ctypes.POINTER(sz)]
        lib.fcr_lstm_workspace_size.restype = i32
        lib.fcr_lstm_forward.argtypes = [ctypes.POINTER(FcrDims), ctypes.POINTER(FcrWeights), vp, vp, i32, vp, sz, vp]
        lib.fcr_lstm_forward.restype = i32
        lib.fcr_lstm_backward.argtypes = [ctypes.POINTER(FcrDims), ctypes.POINTER(FcrWeights), vp,
                                          ctypes.POINTER(vp), ctypes.POINTER(vp), vp, vp, vp, vp, sz, vp]
        lib.fcr_lstm_backward.restype = i32
        lib.fcr_closed_loop_run.argtypes = [ctypes.POINTER(FcrClosedLoop), vp]
        lib.fcr_closed_loop_run.restype = i32
        lib.fcr_window_gather.argtypes = [ctypes.POINTER(FcrWindows), i32, vp, vp, vp, vp, vp, vp]
        lib.fcr_window_gather.restype = i32
        lib.fcr_fnn_workspace_size.argtypes = [i32, i32, ctypes.POINTER(sz)]
        lib.fcr_fnn_workspace_size.restype = i32
        lib.fcr_fnn_forward.argtypes = [i32, i32, i32, vp, vp, vp, vp, vp, vp]
        lib.fcr_fnn_forward.restype = i32
        lib.fcr_fnn_backward.argtypes = [i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, sz, vp]
        lib.fcr_fnn_backward.restype = i32
        lib.fcr_set_small_batch_limit.argtypes = [i32]
        lib.fcr_set_small_batch_limit.restype = i32
        lib.fcr_get_small_batch_limit.argtypes = []
        lib.fcr_get_small_batch_limit.restype = i32
        lib.fcr_set_small_pipe_limit.argtypes = [i32]
        lib.fcr_set_small_pipe_limit.restype = i32
        lib.fcr_get_small_pipe_limit.argtypes = []
        lib.fcr_get_small_pipe_limit.restype = i32
        lib.fcr_set_small_pipe_sets.argtypes = [i32]
        lib.fcr_set_small_pipe_sets.restype = i32
        lib.fcr_get_small_pipe_sets.argtypes = []
        lib.fcr_get_small_pipe_sets.restype = i32
        lib.fcr_set_wide_keep_budget.argtypes = [ctypes.c_int64]
        lib.fcr_set_wide_keep_budget.restype = ctypes.c_int64
        lib.fcr_get_wide_keep_budget.argtypes = []
        lib.fcr_get_wide_keep_budget.restype = ctypes.c_int64
        lib.fcr_last_error.argtypes = []
        lib.fcr_last_error.restype = ctypes.c_char_p
        lib.fcr_abi_version.argtypes = []
        lib.fcr_abi_version.restype = i32
        lib.fcr_wide_bwd_cell_workspace.argtypes = [i32, i32, i32, ctypes.POINTER(sz)]
        lib.fcr_wide_bwd_cell_workspace.restype = i32
        lib.fcr_wide_bwd_cell.argtypes = [i32, i32, i32] + [vp] * 11 + [sz, vp]
        lib.fcr_wide_bwd_cell.restype = i32
        if lib.fcr_abi_version() != ABI_VERSION:
            raise NativeError(f"libfcr ABI {lib.fcr_abi_version()} != expected {ABI_VERSION}")
        _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != FCR_OK:
        msg = load().fcr_last_error().decode(errors="replace")
        raise NativeError(f"{what} failed ({ERRORS.get(rc, rc)}): {msg}")


def set_small_batch_limit(max_batch: int) -> int:
    """fcr_set_small_batch_limit: the process-wide DEFAULT small-batch limit (B <= it runs the small-batch kernels,
    0 = never) of calls whose options inherit it; returns the old value. Per call: MPCLoss(small_batch_limit=...)."""
    return int(load().fcr_set_small_batch_limit(int(max_batch)))


def small_batch_limit() -> int:
    """The process-wide default small-batch limit (fcr_get_small_batch_limit: read-only)."""
    return int(load().fcr_get_small_batch_limit())


def set_small_pipe_limit(max_batch: int) -> int:
    """fcr_set_small_pipe_limit: B <= it (and <= 32 groups) runs the small-batch family's layer-pipelined geometry
    (csrc/fcr_pipe.h), 0 = never; process-wide; returns the old value."""
    return int(load().fcr_set_small_pipe_limit(int(max_batch)))


def small_pipe_limit() -> int:
    """The process-wide layer-pipelined small-batch limit (fcr_get_small_pipe_limit: read-only)."""
    return int(load().fcr_get_small_pipe_limit())


def set_small_pipe_sets(sets: int) -> int:
    """fcr_set_small_pipe_sets: caps the pipelined geometry's window sets (forward <= 4, backward <= 3; 0 = the most
    that fit); process-wide; returns the old value. Results are bit-identical for every value."""
    return int(load().fcr_set_small_pipe_sets(int(sets)))


def small_pipe_sets() -> int:
    """The process-wide window-set setting (fcr_get_small_pipe_sets: read-only; 0 = automatic)."""
    return int(load().fcr_get_small_pipe_sets())


def set_wide_keep_budget(nbytes: int) -> int:
    """fcr_set_wide_keep_budget (H > 52): the process-wide DEFAULT bytes of kept windows a backward-enabled workspace
    may add, so their backward skips the recompute (< 0 = the library's policy: half the device memory free at its
    first sizing, at most 40 % of the device; 0 = none); returns the old budget. Per call: MPCLoss(wide_keep_budget=...)."""
    return int(load().fcr_set_wide_keep_budget(int(nbytes)))


def wide_keep_budget() -> int:
    """The process-wide default keep budget (fcr_get_wide_keep_budget: read-only)."""
    return int(load().fcr_get_wide_keep_budget())


KERNEL_FAMILIES = {0: None, 1: "small", 2: "fused", 3: "wide"}


def workspace_bytes(dims: FcrDims, with_backward: bool, opts: FcrOptions | None = None) -> int:
    out = ctypes.c_size_t(0)
    check(load().fcr_workspace_size(ctypes.byref(dims), ctypes.byref(opts) if opts is not None else None,
                                    int(bool(with_backward)), ctypes.byref(out)), "fcr_workspace_size")
    return int(out.value)


def kept_windows(dims: FcrDims, ws_bytes: int) -> int:
    """fcr_wide_kept_windows: windows (of N) a backward-enabled H > 52 workspace of ws_bytes keeps."""
    out = ctypes.c_int32(0)
    check(load().fcr_wide_kept_windows(ctypes.byref(dims), int(ws_bytes), ctypes.byref(out)), "fcr_wide_kept_windows")
    return int(out.value)
