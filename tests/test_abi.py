"""CPU-side checks of the drop-in boundary: libxdrgpu.so loads, exports every
symbol include/xdrg.h declares, the ctypes mirror matches the header, and the
host-only schema compiler enforces the rpcgen vocabulary (no GPU needed)."""
import ctypes
import os
import re

import pytest

from oncrpc4j_amd import abi, engine
from oncrpc4j_amd.columns import field_xdr_bytes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "xdrg.h")


def _header():
    with open(HEADER) as f:
        return f.read()


def test_header_functions_exported():
    decl = set(re.findall(r"^\s*(?:int|uint64_t|const char \*)\s*\*?(xdrg_\w+)\s*\(", _header(), re.M))
    assert decl, "no declarations parsed"
    lib = engine.lib()
    for name in decl:
        assert hasattr(lib, name), f"{name} not exported"
    assert decl == set(abi.FUNCTIONS), "abi.FUNCTIONS out of sync with include/xdrg.h"


def test_header_constants_match_mirror():
    defs = dict(re.findall(r"#define\s+(XDRG_\w+)\s+(0x[0-9a-fA-F]+u?|\d+)", _header()))
    val = {k: int(v.rstrip("u"), 0) for k, v in defs.items()}
    assert val["XDRG_ABI_VERSION"] == abi.ABI_VERSION
    for name in ("OK", "E_SHORT", "E_CORRUPT", "E_FIXED_LEN", "E_CAPACITY", "E_FRAME", "E_INVAL",
                 "E_HIP", "E_NOMEM", "E_INCOMPLETE", "FRAME_RM", "ASYNC", "CTX_TIMING",
                 "KERNEL_FIXED_ENCODE", "KERNEL_VAR_DECODE", "KERNEL_FRAME_SCAN", "KERNEL_COUNT"):
        assert val["XDRG_" + name] == getattr(abi, name), name
    for t in ("INT", "UINT", "ENUM", "BOOL", "HYPER", "UHYPER", "FLOAT", "DOUBLE", "SHORT", "BYTE",
              "OPAQUE", "STRING"):
        assert val["XDRG_T_" + t] == getattr(abi, "T_" + t)
    for k in ("SCALAR", "FIXED", "DYNAMIC"):
        assert val["XDRG_K_" + k] == getattr(abi, "K_" + k)


def test_struct_layouts():
    assert ctypes.sizeof(abi.Field) == 16
    assert ctypes.sizeof(abi.Column) == 32


def test_status_strings_match_reference_messages():
    L = engine.lib()
    assert L.xdrg_abi_version() == abi.ABI_VERSION
    assert L.xdrg_status_string(abi.E_SHORT) == b"xdr stream too short"     # Xdr.java:1030
    assert L.xdrg_status_string(abi.E_CORRUPT) == b"corrupted xdr"          # Xdr.java:1036


GOOD = [
    [(abi.T_INT, abi.K_SCALAR, 0)] * 8,
    [(abi.T_INT, abi.K_SCALAR, 0), (abi.T_STRING, abi.K_DYNAMIC, 0), (abi.T_INT, abi.K_DYNAMIC, 0)],
    [(abi.T_OPAQUE, abi.K_FIXED, 5), (abi.T_HYPER, abi.K_FIXED, 3), (abi.T_BOOL, abi.K_SCALAR, 0)],
    [(abi.T_DOUBLE, abi.K_SCALAR, 0), (abi.T_SHORT, abi.K_FIXED, 3), (abi.T_BYTE, abi.K_DYNAMIC, 0)],
]
BAD = [
    [(abi.T_BOOL, abi.K_FIXED, 3)],        # rpcgen emits no boolean vectors
    [(abi.T_STRING, abi.K_FIXED, 8)],      # strings are string<> only
    [(abi.T_OPAQUE, abi.K_SCALAR, 0)],     # opaque needs [N] or <>
    [(99, abi.K_SCALAR, 0)],
    [(abi.T_INT, 7, 0)],
]


@pytest.mark.parametrize("fields", GOOD)
def test_schema_compile(fields):
    s = engine.Schema(fields)
    fixed = all(k != abi.K_DYNAMIC for _, k, _ in fields)
    want = sum(field_xdr_bytes(f) for f in fields) if fixed else 0
    assert s.fixed_size == want


@pytest.mark.parametrize("fields", BAD)
def test_schema_rejects(fields):
    with pytest.raises(engine.XdrgError) as ei:
        engine.Schema(fields)
    assert ei.value.code == abi.E_INVAL


def test_reserved_must_be_zero():
    arr = (abi.Field * 1)()
    arr[0].type, arr[0].kind, arr[0].count, arr[0].reserved = abi.T_INT, abi.K_SCALAR, 0, 1
    h = ctypes.c_void_p()
    assert engine.lib().xdrg_schema_create(arr, 1, ctypes.byref(h)) == abi.E_INVAL
