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


# Every entry point whose work is empty (a zero count) returns MVR_OK before it looks at the pointers of the empty
# arrays, which may be NULL (mvreg.h conventions) — a zero-element torch tensor's data_ptr() is 0.  These calls
# return before any HIP call, so they run without a GPU.  (Round 5's GPU suite failed on exactly this ordering in
# mvr_radix_sort_pairs.)
_Z = None      # NULL
_EMPTY_CALLS = {
    "mvr_radix_sort_pairs": lambda L: L.mvr_radix_sort_pairs(_Z, _Z, 0, 64, _Z, _Z, 0, _Z),
    "mvr_kernel_map_order": lambda L: L.mvr_kernel_map_order(_Z, _Z, 1, 0, 27, _Z, _Z, 0, _Z),
    "mvr_kernel_map_x": lambda L: L.mvr_kernel_map_x(_Z, 0, _Z, 0, 3, 1, 0, _Z, _Z, _Z),
    "mvr_kernel_map_sym": lambda L: L.mvr_kernel_map_sym(_Z, 0, _Z, 0, 1, _Z, _Z),
    "mvr_kernel_map_transpose": lambda L: L.mvr_kernel_map_transpose(_Z, 0, 27, _Z, 0, _Z),
    "mvr_kernel_map": lambda L: L.mvr_kernel_map(_Z, 0, _Z, 0, 3, 1, 1, _Z, _Z),
    "mvr_spconv_x": lambda L: L.mvr_spconv_x(_Z, 32, 32, _Z, _Z, 27, 0, _Z, 32, _Z, _bn0(), 1e-5, _Z, 0, 1, _Z, 32,
                                             _Z, _Z, _Z, _Z, _Z),
    "mvr_spconv": lambda L: L.mvr_spconv(_Z, 32, 32, _Z, _Z, 27, 0, _Z, 32, _Z, _bn0(), 1e-5, _Z, 0, 1, _Z, 32, _Z,
                                         _Z, _Z),
    "mvr_spconv_c1_x": lambda L: L.mvr_spconv_c1_x(_Z, 0, _Z, 0, 0, _Z, 7, 1, _Z, 32, _bn0(), 1e-5, 1, _Z, 32, _Z,
                                                   _Z),
    "mvr_l2norm_rows": lambda L: L.mvr_l2norm_rows(_Z, 0, 32, 32, _Z),
    "mvr_feat_nn": lambda L: L.mvr_feat_nn(_Z, 0, _Z, 0, _Z, 0, _Z, 0, _Z, 0, 5000, 5000, 32, 1.0, 0, _Z, 0, 0, _Z,
                                           _Z),
    "mvr_feat_nn_ws": lambda L: L.mvr_feat_nn_ws(_Z, 0, _Z, 0, _Z, 0, _Z, 0, _Z, 3, 0, 5000, 32, 1.0, 0, _Z, 0, 0,
                                                 _Z, 0, _Z, 0, _Z),
    "mvr_feat_nn_gumbel": lambda L: L.mvr_feat_nn_gumbel(_Z, 0, _Z, 0, _Z, 0, _Z, 0, _Z, 0, 5000, 5000, 32, 1.0, 1, 7,
                                                         _Z, 0, 0, _Z, _Z),
    "mvr_feat_knn2": lambda L: L.mvr_feat_knn2(_Z, 0, _Z, 0, _Z, 0, 100, 100, 32, _Z, _Z, _Z),
    "mvr_gather_rows": lambda L: L.mvr_gather_rows(_Z, 32, _Z, 0, _Z, _Z),
    "mvr_fps": lambda L: L.mvr_fps(_Z, _Z, _Z, 0, 5000, _Z, _Z),
    "mvr_xs_to_channels": lambda L: L.mvr_xs_to_channels(_Z, 0, 6, 6, 0, 5000, _Z, 0, 5000, _Z),
    "mvr_procrustes": lambda L: L.mvr_procrustes(_Z, _Z, 0, 6, _Z, 0, _Z, _Z, 0, 0, 5000, 1, 1e-6, _Z, _Z, _Z, 0, _Z,
                                                 0, _Z, 0, _Z),
    "mvr_procrustes_f64": lambda L: L.mvr_procrustes_f64(_Z, _Z, 0, 6, _Z, 0, _Z, _Z, 0, 0, 5000, 1, 1e-6, _Z, _Z,
                                                         _Z, 0, _Z, 0, _Z, 0, _Z),
    "mvr_ransac": lambda L: L.mvr_ransac(_Z, _Z, 0, _Z, 0, 4, 2500, 0.05, 0, _Z, _Z, _Z, _Z, _Z, _Z, 0, _Z),
    "mvr_knn1": lambda L: L.mvr_knn1(_Z, 0, 3, _Z, 0, 3, 0, 100, 100, _Z, _Z, _Z),
    "mvr_mutuals": lambda L: L.mvr_mutuals(_Z, 0, 3, _Z, 0, 3, _Z, 0, 3, _Z, 0, 3, 0, 100, 0.01, _Z, _Z, _Z),
    "mvr_oan_diff_pool": lambda L: L.mvr_oan_diff_pool(_Z, 0, 5000, _Z, _Z, 0, _Z, _Z, 0, 128, 5000, 500, _Z, 0, 500,
                                                       _Z, 0, 0, _Z),
    "mvr_oan_diff_pool_ws": lambda L: L.mvr_oan_diff_pool_ws(_Z, 0, 5000, _Z, _Z, 0, _Z, _Z, 0, 128, 5000, 500, _Z,
                                                             0, 500, _Z, 0, 0, _Z, 0, _Z),
    "mvr_oan_diff_unpool": lambda L: L.mvr_oan_diff_unpool(_Z, 0, 5000, _Z, _Z, 0, _Z, _Z, _Z, 0, 500, 0, 128, 5000,
                                                           500, _Z, 0, 5000, _Z, 0, 0, _Z, 0, _Z),
    "mvr_oaf_conv2_f32": lambda L: L.mvr_oaf_conv2_f32(128, 500, 500, 0, _Z, 0, 500, _Z, 500, _Z, 0, 500, _Z, 0, _Z,
                                                       _Z, _Z, 0, _Z, 0, _Z, 0, _Z),
    "mvr_gemm_f32": lambda L: L.mvr_gemm_f32(128, 0, 128, 1, _Z, 0, 128, _Z, 0, 128, 0, _Z, 0, 128, _Z, 0, _Z, 0, _Z,
                                             _Z, 0, 0, 0, _Z, 0, 0, 0, 1, _Z, _Z),
    "mvr_oan_block_forward": lambda L: L.mvr_oan_block_forward(_Z, _Z, 0, 5000, _Z, 0, 6, 0, 5000, 0, _Z, _Z, _Z, _Z,
                                                               _Z, _Z, _Z, _Z, 0, _Z, _Z, 0, _Z, 0, _Z),
    "mvr_sample_rand_mt19937": lambda L: L.mvr_sample_rand_mt19937(_Z, _Z, _Z, 0, 5000, _Z, _Z),
    "mvr_radius_overlap_count": lambda L: L.mvr_radius_overlap_count(_Z, 0, _Z, _Z, 2, 0, _Z, _Z, 0, 0, 0.05, _Z,
                                                                     _Z),
}


def _bn0():
    from lib import _native
    return _native.BnP()


@pytest.mark.skipif(not os.path.exists(LIB), reason="libmvreg_hip.so not built")
@pytest.mark.parametrize("name", sorted(_EMPTY_CALLS))
def test_empty_count_accepts_null_pointers(name):
    from lib import _native
    L = _native.lib()
    assert _EMPTY_CALLS[name](L) == 0, name


@pytest.mark.skipif(not os.path.exists(LIB), reason="libmvreg_hip.so not built")
def test_kernel_map_orders_all_maps_empty():
    from lib import _native
    L = _native.lib()
    n = 3
    Mo = (ctypes.c_int64 * n)(0, 0, 0)
    nbr = (ctypes.c_void_p * n)(None, None, None)
    steps = (ctypes.c_int * n)(1, 2, 4)
    assert L.mvr_kernel_map_orders(n, nbr, None, steps, Mo, 27, None, None, 0, None) == 0
    # a non-empty map still needs its table and the output / workspace pointers
    Mo[1] = 5
    assert L.mvr_kernel_map_orders(n, nbr, None, steps, Mo, 27, None, None, 0, None) == -1


@pytest.mark.skipif(not os.path.exists(LIB), reason="libmvreg_hip.so not built")
def test_nonempty_calls_still_reject_null_pointers():
    from lib import _native
    L = _native.lib()
    assert L.mvr_radix_sort_pairs(None, None, 10, 64, None, None, 0, None) == -1
    assert L.mvr_kernel_map_x(None, 10, None, 0, 3, 1, 0, None, None, None) == -1
    assert L.mvr_l2norm_rows(None, 10, 32, 32, None) == -1
    assert L.mvr_feat_nn(None, 0, None, 0, None, 0, None, 0, None, 1, 5000, 5000, 32, 1.0, 0, None, 0, 0, None,
                         None) == -1
    # scalar arguments are validated before the empty short-cut
    assert L.mvr_radix_sort_pairs(None, None, 0, 65, None, None, 0, None) == -1
    assert L.mvr_radix_sort_pairs(None, None, -1, 64, None, None, 0, None) == -1
