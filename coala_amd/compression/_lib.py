"""ctypes binding of the codec's C ABI (include/coalac.h) — the only way the host side reaches the GPU.

There is deliberately no CPU fallback: if the HIP library is missing or cannot be loaded, every codec
call raises. (The CPU oracle under oracle/ is test infrastructure and is never imported from here.)
"""
import ctypes
import os
import threading

from .. import _build

COALAC_FLAG_FORCE_EXACT = 1
COALAC_FLAG_GENERIC_SELECT = 2
COALAC_FLAG_STAMPS = 4
COALAC_FLAG_NO_FORK = 8
COALAC_AGG_DIV = 0     # acc / total            (torch CPU division by a scalar)
COALAC_AGG_RECIP = 1   # acc * (1.0f / total)   (torch GPU division by a host scalar)
COALAC_AGG_SUM = 2     # acc                    (weighted_sum: the multi-GPU per-rank sum)

ERRORS = {
    -1: "COALAC_EINVAL",
    -2: "COALAC_EBITS",
    -3: "COALAC_EWORKSPACE",
    -4: "COALAC_EHIP",
    -5: "COALAC_EDEVICE",
    -6: "COALAC_ENOMEM",
}

# every symbol include/coalac.h declares: (name, restype, argtypes)
_P = ctypes.c_void_p
_U64 = ctypes.c_uint64
_I = ctypes.c_int
SIGNATURES = [
    ("coalac_version", _I, []),
    ("coalac_last_error", ctypes.c_char_p, []),
    ("coalac_plan_create", _I, [_P, _I, _I, ctypes.POINTER(_P)]),
    ("coalac_plan_destroy", _I, [_P]),
    ("coalac_plan_query", _I, [_P, ctypes.POINTER(_U64), ctypes.POINTER(_U64), ctypes.POINTER(_U64),
                               ctypes.POINTER(_U64)]),
    # encode: plan, in / seg pointers, base, idx, vals, mn, scale, ustart, ws, ws_bytes, flags, stream (+ events)
    ("coalac_encode", _I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _U64, ctypes.c_uint, _P]),
    ("coalac_encode_segptr", _I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _U64, ctypes.c_uint, _P]),
    # decode: plan, idx, vals, mn, scale, ustart, base, out, stream (+ events)
    ("coalac_decode", _I, [_P, _P, _P, _P, _P, _P, _P, _P, _P]),
    ("coalac_encode_ev", _I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _U64, ctypes.c_uint, _P, _P]),
    ("coalac_decode_ev", _I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    # aggregate: plan, clients, idx, vals, mn, scale, ustart, weights, total, mode, mask, base, out, stream (+ events)
    ("coalac_aggregate", _I, [_P, _I, _P, _P, _P, _P, _P, _P, ctypes.c_float, _I, _P, _P, _P, _P]),
    ("coalac_aggregate_ev", _I, [_P, _I, _P, _P, _P, _P, _P, _P, ctypes.c_float, _I, _P, _P, _P, _P, _P]),
    ("coalac_gather", _I, [_P, _I, _I, _P, _P]),
    ("coalac_workspace_fallbacks", _I, [_P, _P, _P, ctypes.POINTER(_I)]),
    ("coalac_debug_stamps", _I, [_P, _P, _P, ctypes.POINTER(ctypes.c_uint64), _I]),
    ("coalac_debug_brackets", _I, [_P, _P, _P, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32), _I]),
]

ABI_VERSION = 5


class CodecError(RuntimeError):
    pass


class SegDesc(ctypes.Structure):
    _fields_ = [("in_off", _U64), ("n", _U64), ("k", _U64), ("out_off", _U64)]


_lock = threading.Lock()
_lib = None


def lib_path():
    """The in-tree library; COALAC_LIB names another build of the same source (A/B variants under tools/)."""
    return os.environ.get("COALAC_LIB") or _build.LIB


def load(build_if_missing=True):
    """Load libcoalac.so (building it first if it is missing and hipcc is available)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = lib_path()
        if not os.environ.get("COALAC_LIB") and (
                not os.path.exists(path) or (build_if_missing and _build.stale() and _can_build())):
            if not build_if_missing:
                raise CodecError(f"HIP codec library not found at {path}; run __graft_entry__.build()")
            _build.build()
        lib = ctypes.CDLL(path)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.coalac_version()
        if v != ABI_VERSION:
            raise CodecError(f"libcoalac ABI version {v} != expected {ABI_VERSION}")
        _lib = lib
        return lib


def _can_build():
    try:
        _build.hipcc()
        return True
    except RuntimeError:
        return False


def check(rc, what):
    if rc != 0:
        msg = _lib.coalac_last_error().decode(errors="replace") if _lib is not None else ""
        raise CodecError(f"{what} failed: {ERRORS.get(rc, rc)}: {msg}")
