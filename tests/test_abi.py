"""The C-ABI library builds/loads without a GPU, exports every symbol include/coalac.h declares, and
validates plans before touching the device. No compute calls here (no GPU in CI)."""
import ctypes
import re

import pytest

from coala_amd import _build
from coala_amd.compression import _lib


def declared_symbols():
    hdr = open(_build.HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(coalac_\w+)\s*\(", hdr, re.M)))


def test_header_and_binding_agree():
    names = declared_symbols()
    assert len(names) >= 10
    assert sorted(n for n, _, _ in _lib.SIGNATURES) == names


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.coalac_version() == _lib.ABI_VERSION


def _create(segs, bits=8):
    lib = _lib.load()
    arr = (_lib.SegDesc * len(segs))(*[_lib.SegDesc(*s) for s in segs])
    h = ctypes.c_void_p()
    rc = lib.coalac_plan_create(arr, len(segs), bits, ctypes.byref(h))
    return rc, lib.coalac_last_error().decode()


@pytest.mark.parametrize("segs,bits,code,msg", [
    ([(0, 10, 1, 0)], 9, -2, "bits"),
    ([(2, 10, 1, 0)], 8, -1, "multiple of 4"),
    ([(0, 10, 0, 0)], 8, -1, "k="),
    ([(0, 10, 11, 0)], 8, -1, "k="),
    ([(0, 0, 1, 0)], 8, -1, "k="),
    ([(0, 10, 2, 0), (8, 10, 2, 2)], 8, -1, "input ranges overlap"),
    ([(0, 10, 2, 0), (16, 10, 2, 1)], 8, -1, "output ranges overlap"),
    ([(0, 1 << 31, 1, 0)], 8, -1, ">= 2^31"),
])
def test_plan_validation(segs, bits, code, msg):
    rc, err = _create(segs, bits)
    assert rc == code and msg in err


def test_null_arguments():
    lib = _lib.load()
    assert lib.coalac_plan_create(None, 1, 8, None) == -1
    assert lib.coalac_plan_destroy(None) == 0
    assert lib.coalac_encode(None, None, None, None, None, None, None, None, None, 0, 0, None) == -1
    assert lib.coalac_decode(None, None, None, None, None, None, None, None, None, 0, None) == -1


def test_binding_argument_counts_match_header():
    """Every declaration's parameter count equals the ctypes binding's (an ABI change that misses one side would
    shift every argument after it)."""
    hdr = re.sub(r"/\*.*?\*/", "", open(_build.HDR).read(), flags=re.S)
    decls = dict(re.findall(r"(coalac_\w+)\s*\(([^;{]*?)\)\s*;", hdr))
    for name, _, args in _lib.SIGNATURES:
        params = decls[name].strip()
        n = 0 if params in ("", "void") else params.count(",") + 1
        assert n == len(args), (name, n, len(args))


def test_enum_constants_match_header():
    """Every COALAC_FLAG_* / COALAC_AGG_* value the Python binding uses is the header's (ABI 5: no stage enums)."""
    hdr = open(_build.HDR).read()
    declared = {k: int(v) for k, v in re.findall(r"\b(COALAC_(?:FLAG|STAGE|AGG)_\w+)\s*=\s*(\d+)", hdr)}
    assert {"COALAC_FLAG_FORCE_EXACT", "COALAC_FLAG_NO_FORK", "COALAC_AGG_DIV", "COALAC_AGG_SUM"} <= set(declared)
    assert not any(k.startswith("COALAC_STAGE_") for k in declared)
    for name, value in declared.items():
        assert getattr(_lib, name) == value, name
