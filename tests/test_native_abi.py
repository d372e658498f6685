"""CPU-side checks of the C ABI: the library (built by __graft_entry__.build())
loads and exports every symbol include/mvreg.h declares.  No compute calls."""
import ctypes
import os
import re

import pytest

from conftest import ROOT, PKG

LIB = os.path.join(PKG, "libmvreg_hip.so")
HDR = os.path.join(ROOT, "include", "mvreg.h")


def header_symbols():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t)\s+(mvr_\w+)\s*\(", txt, re.M)))


def test_header_declares_symbols():
    syms = header_symbols()
    assert "mvr_procrustes" in syms and "mvr_oan_block_forward" in syms


@pytest.mark.skipif(not os.path.exists(LIB), reason="libmvreg_hip.so not built")
def test_library_exports_every_header_symbol():
    import torch  # noqa: F401  (bind to torch's HIP runtime first, as the product path does)
    L = ctypes.CDLL(LIB)
    missing = [s for s in header_symbols() if not hasattr(L, s)]
    assert not missing, missing


@pytest.mark.skipif(not os.path.exists(LIB), reason="libmvreg_hip.so not built")
def test_python_binding_covers_header():
    from lib import _native
    assert set(header_symbols()) == set(_native.EXPORTS)
    L = _native.lib()
    assert L.mvr_oan_block_workspace_bytes(128, 500, 6, 2, 5000) > 2 * 5000 * 128 * 4


@pytest.mark.skipif(not os.path.exists(LIB), reason="libmvreg_hip.so not built")
def test_native_structs_match_header_layout():
    from lib import _native as N
    # 4 ints + conv + 3 arrays of 8 PointCN/OAFilter + 2 (bn,conv) + conv
    ptr = ctypes.sizeof(ctypes.c_void_p)
    conv, bn = 2 * ptr, 4 * ptr
    pcn = bn + conv + bn + conv + conv
    oaf = 3 * (bn + conv)
    want = 16 + conv + 8 * pcn + bn + conv + 8 * oaf + bn + conv + 8 * pcn + conv
    assert ctypes.sizeof(N.OanBlockP) == want
