"""ctypes binding of libmvreg_hip.so (the C ABI declared in include/mvreg.h).

The product path has NO CPU fallback: if the HIP library or a HIP device is
missing, every op raises.  torch is imported first so that the library binds
to the HIP runtime torch already loaded (one runtime, shared streams).
"""
import ctypes
import os

import torch

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MVR_LIB") or os.path.join(_PKG, "libmvreg_hip.so")   # MVR_LIB: tools' variant builds
_lib = None

c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_float = ctypes.c_float
c_vp = ctypes.c_void_p
c_size = ctypes.c_size_t


class ConvP(ctypes.Structure):
    _fields_ = [("weight", c_vp), ("bias", c_vp)]


class BnP(ctypes.Structure):
    _fields_ = [("gamma", c_vp), ("beta", c_vp), ("mean", c_vp), ("var", c_vp)]


class PointCNP(ctypes.Structure):
    _fields_ = [("bn1", BnP), ("conv3", ConvP), ("bn5", BnP), ("conv7", ConvP), ("shortcut", ConvP)]


class OAFilterP(ctypes.Structure):
    _fields_ = [("bn1", BnP), ("conv1", ConvP), ("bn2", BnP), ("conv2", ConvP), ("bn3", BnP), ("conv3", ConvP)]


MAX_HALF = 8


class OanBlockP(ctypes.Structure):
    _fields_ = [("in_channels", c_int), ("channels", c_int), ("clusters", c_int), ("half_layers", c_int),
                ("conv1", ConvP), ("l1_1", PointCNP * MAX_HALF), ("down_bn", BnP), ("down_conv", ConvP),
                ("l2", OAFilterP * MAX_HALF), ("up_bn", BnP), ("up_conv", ConvP), ("l1_2", PointCNP * MAX_HALF),
                ("output", ConvP)]


_SIGS = {
    "mvr_procrustes": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_float,
                               c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_int, c_vp]),
    "mvr_procrustes_f64": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_int, c_int, c_int,
                                   ctypes.c_double, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_int, c_vp]),
    "mvr_ransac_workspace_bytes": (c_size, [c_int, c_int]),
    "mvr_ransac": (c_int, [c_vp, c_vp, c_i64, c_vp, c_int, c_int, c_int, ctypes.c_double, ctypes.c_uint64, c_vp, c_vp,
                           c_vp, c_vp, c_vp, c_vp, c_size, c_vp]),
    "mvr_gemm_f32": (c_int, [c_int, c_int, c_int, c_int, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_int, c_vp, c_i64,
                             c_i64, c_vp, c_i64, c_vp, c_int, c_vp, c_vp, c_i64, c_i64, c_int, c_vp, c_i64, c_int,
                             c_int, c_int, c_vp, c_vp]),
    "mvr_oaf_conv2_f32": (c_int, [c_int, c_int, c_int, c_int, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64,
                                  c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "mvr_oaf_conv2_image_bytes": (c_size, [c_int, c_int]),
    "mvr_oan_block_workspace_bytes": (c_size, [c_int, c_int, c_int, c_int, c_int]),
    "mvr_set_math": (c_int, [c_int]),
    "mvr_debug_force": (c_int, [c_int, c_int]),
    "mvr_attn_reruns": (c_int, [c_int]),
    "mvr_debug_stage_hash": (c_int, [c_vp, c_int]),
    "mvr_debug_stage_dump": (c_int, [c_int, c_vp, c_size]),
    "mvr_oan_diff_pool": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_int, c_int, c_int, c_int,
                                  c_vp, c_i64, c_i64, c_vp, c_i64, c_int, c_vp]),
    "mvr_oan_diff_pool_ws": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_int, c_int, c_int, c_int,
                                  c_vp, c_i64, c_i64, c_vp, c_i64, c_int, c_vp, c_size, c_vp]),
    "mvr_oan_diff_pool_workspace_bytes": (c_size, [c_int, c_int, c_int]),
    "mvr_oan_diff_unpool_workspace_bytes": (c_size, [c_int, c_int, c_int]),
    "mvr_oan_diff_unpool": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_i64, c_int,
                                    c_int, c_int, c_int, c_vp, c_i64, c_i64, c_vp, c_i64, c_int, c_vp, c_size, c_vp]),
    "mvr_oan_block_forward": (c_int, [ctypes.POINTER(OanBlockP), c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_int, c_int, c_int,
                                      c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_int, c_vp,
                                      c_size, c_vp]),
    "mvr_feat_nn": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_int, c_int, c_int, c_int,
                            c_float, c_int, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "mvr_feat_nn_gumbel": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_int, c_int, c_int,
                                   c_int, c_float, c_int, ctypes.c_uint64, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "mvr_feat_nn_workspace_bytes": (c_size, [c_int, c_int]),
    "mvr_feat_nn_ws": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_int, c_int, c_int, c_int,
                               c_float, c_int, c_vp, c_i64, c_i64, c_vp, c_int, c_vp, c_size, c_vp]),
    "mvr_gather_rows": (c_int, [c_vp, c_int, c_vp, c_int, c_vp, c_vp]),
    "mvr_sample_rand_mt19937": (c_int, [c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp]),
    "mvr_feat_knn2": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp]),
    "mvr_fps": (c_int, [c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp]),
    "mvr_knn1": (c_int, [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_int, c_int, c_int, c_vp, c_vp, c_vp]),
    "mvr_mutuals": (c_int, [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_int,
                            c_int, c_float, c_vp, c_vp, c_vp]),
    "mvr_voxel_centroids_workspace_bytes": (c_size, [c_i64]),
    "mvr_voxel_centroids": (c_int, [c_vp, c_vp, c_int, c_i64, ctypes.c_double, c_vp, c_size, c_vp, c_vp, c_vp]),
    "mvr_radius_index_bytes": (c_size, [c_i64]),
    "mvr_radius_index_build": (c_int, [c_vp, c_vp, c_int, c_i64, ctypes.c_double, c_vp, c_size, c_vp]),
    "mvr_radius_overlap_count": (c_int, [c_vp, c_size, c_vp, c_vp, c_int, c_i64, c_vp, c_vp, c_int, c_i64,
                                         ctypes.c_double, c_vp, c_vp]),
    "mvr_hash_table_bytes": (c_size, [c_i64]),
    "mvr_voxelize_workspace_bytes": (c_size, [c_i64]),
    "mvr_voxelize_hint_workspace_bytes": (c_size, [c_i64, c_i64]),
    "mvr_voxelize_hint": (c_int, [c_vp, c_vp, c_int, c_i64, ctypes.c_double, c_i64, c_vp, c_size, c_vp, c_vp, c_vp,
                                  c_vp]),
    "mvr_voxelize": (c_int, [c_vp, c_vp, c_int, c_i64, ctypes.c_double, c_vp, c_size, c_vp, c_vp, c_vp, c_vp]),
    "mvr_voxelize_f64": (c_int, [c_vp, c_vp, c_int, c_i64, ctypes.c_double, c_vp, c_size, c_vp, c_vp, c_vp, c_vp]),
    "mvr_coords_downsample_workspace_bytes": (c_size, [c_i64]),
    "mvr_coords_downsample": (c_int, [c_vp, c_i64, c_int, c_int, c_vp, c_size, c_vp, c_vp, c_vp]),
    "mvr_hash_build": (c_int, [c_vp, c_i64, c_vp, c_size, c_vp]),
    "mvr_hash_build_lattice": (c_int, [c_vp, c_i64, c_int, c_vp, c_size, c_vp]),
    "mvr_kernel_map": (c_int, [c_vp, c_i64, c_vp, c_size, c_int, c_int, c_int, c_vp, c_vp]),
    "mvr_kernel_map_x": (c_int, [c_vp, c_i64, c_vp, c_size, c_int, c_int, c_int, c_vp, c_vp, c_vp]),
    "mvr_kernel_map_sym": (c_int, [c_vp, c_i64, c_vp, c_size, c_int, c_vp, c_vp]),
    "mvr_kernel_map_transpose": (c_int, [c_vp, c_i64, c_int, c_vp, c_i64, c_vp]),
    "mvr_kernel_map_order_bytes": (c_size, [c_i64]),
    "mvr_kernel_map_order": (c_int, [c_vp, c_vp, c_int, c_i64, c_int, c_vp, c_vp, c_size, c_vp]),
    "mvr_kernel_map_orders_bytes": (c_size, [c_i64]),
    "mvr_kernel_map_orders": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_size, c_vp]),
    "mvr_radix_sort_pairs_bytes": (c_size, [c_i64]),
    "mvr_radix_sort_pairs": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_size, c_vp]),
    "mvr_spconv": (c_int, [c_vp, c_i64, c_int, c_vp, c_vp, c_int, c_i64, c_vp, c_int, c_vp, BnP, c_float, c_vp, c_i64,
                           c_int, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "mvr_spconv_x": (c_int, [c_vp, c_i64, c_int, c_vp, c_vp, c_int, c_i64, c_vp, c_int, c_vp, BnP, c_float, c_vp,
                             c_i64, c_int, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mvr_spconv_c1_x": (c_int, [c_vp, c_i64, c_vp, c_i64, c_size, c_vp, c_int, c_int, c_vp, c_int, BnP, c_float,
                                c_int, c_vp, c_i64, c_vp, c_vp]),
    "mvr_spconv_wimage_bytes": (c_size, [c_int, c_int, c_int]),
    "mvr_spconv_wimage": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_size, c_vp]),
    "mvr_brick_map_bytes": (c_size, [c_i64]),
    "mvr_brick_map_build": (c_int, [c_vp, c_i64, c_vp, c_size, c_vp]),
    "mvr_brick_map_build_stride": (c_int, [c_vp, c_i64, c_int, c_vp, c_size, c_vp]),
    "mvr_spconv_c1": (c_int, [c_vp, c_i64, c_vp, c_i64, c_size, c_vp, c_int, c_int, c_vp, c_int, BnP, c_float, c_int,
                              c_vp, c_i64, c_vp]),
    "mvr_l2norm_rows": (c_int, [c_vp, c_i64, c_int, c_i64, c_vp]),
    "mvr_prof_set": (c_int, [c_int]),
    "mvr_prof_mask": (c_int, [ctypes.c_uint]),
    "mvr_prof_seq": (c_int, [c_vp, c_vp, c_int]),
    "mvr_prof_get": (c_int, [c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong),
                             ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "mvr_oan_last_layout": (c_int, []),
    "mvr_source_hash": (c_int, [ctypes.c_char_p, c_size]),
    "mvr_xs_to_channels": (c_int, [c_vp, c_i64, c_i64, c_int, c_int, c_int, c_vp, c_i64, c_i64, c_vp]),
}

# every symbol include/mvreg.h declares (checked by tests/test_native_abi.py)
EXPORTS = tuple(_SIGS)


def lib():
    """Load libmvreg_hip.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libmvreg_hip.so not found at %s — run __graft_entry__.build() "
                               "(there is no CPU fallback for the HIP path)" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


_hip_ok = False


def require_hip(t=None):
    global _hip_ok
    if not _hip_ok:   # torch.cuda.is_available() queries the runtime (microseconds): ask once
        if not torch.cuda.is_available():
            raise RuntimeError("mvreg HIP path: no HIP device available (no CPU fallback)")
        _hip_ok = True
    if t is not None and t.device.type != "cuda":
        raise RuntimeError("mvreg HIP path: tensor on %s, expected a HIP device" % t.device)


def stream():
    return c_vp(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    if t is None:
        return None
    return c_vp(t.data_ptr())


def check(rc, name):
    if rc != 0:
        raise RuntimeError("%s failed with code %d" % (name, rc))


def source_hash():
    """The loaded library's source identity (csrc/Makefile SRC_HASH; variant builds append their flags)."""
    buf = ctypes.create_string_buffer(128)
    check(lib().mvr_source_hash(buf, len(buf)), "mvr_source_hash")
    return buf.value.decode()


PROF_KINDS = {"conv_pts": 0, "embed": 1, "pool": 2, "unpool": 3, "oafilter": 4, "small": 5, "procrustes": 6,
              "feat_nn": 7, "spconv": 8, "sparse_misc": 9, "pointcn": 10}


def prof_set(on):
    check(lib().mvr_prof_set(int(on)), "mvr_prof_set")


def prof_mask(kinds=None):
    """Record only these kinds (names or ids; None = all) while profiling is enabled."""
    m = 0xFFFFFFFF if kinds is None else sum(1 << (PROF_KINDS[k] if isinstance(k, str) else int(k)) for k in kinds)
    check(lib().mvr_prof_mask(m), "mvr_prof_mask")


def prof_seq():
    """[(kind name, algorithmic bytes)] of every profiled launch since prof_set(1), in order."""
    import numpy as np
    L = lib()
    n = L.mvr_prof_seq(None, None, 0)
    k = np.zeros(max(n, 1), np.int32)
    b = np.zeros(max(n, 1), np.float64)
    L.mvr_prof_seq(k.ctypes.data, b.ctypes.data, n)
    names = {v: s for s, v in PROF_KINDS.items()}
    return [(names.get(int(k[i]), str(int(k[i]))), float(b[i])) for i in range(n)]


def prof_get(kind):
    """(device ms, launches, algorithmic flops, algorithmic bytes) since prof_set(1)."""
    ms, n, fl, by = ctypes.c_double(), ctypes.c_longlong(), ctypes.c_double(), ctypes.c_double()
    k = PROF_KINDS[kind] if isinstance(kind, str) else int(kind)
    check(lib().mvr_prof_get(k, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl), ctypes.byref(by)),
          "mvr_prof_get")
    return ms.value, n.value, fl.value, by.value


MATH_KERNELS = "pconv_math,attn_math,spconv_math,gemm_f16,feat_nn"   # the kernels mvr_set_math(1) switches
# mvr_debug_force paths (include/mvreg.h, csrc/knobs.hpp ForcePath)
FORCE = {"feat_nn_online": 0, "generic_gemm": 1, "unfused_attn": 2, "no_conv1_fold": 3, "pool_nosplit": 4,
         "unpool8": 5, "row_layout": 6}


def math_state():
    """The library's arithmetic as it is set now: 0 f32eq, 1 split16 (read back: mvr_set_math returns the previous
    mode)."""
    L = lib()
    m = L.mvr_set_math(0)
    L.mvr_set_math(m)
    return m


def set_math(mode):
    """Select the MFMA operand arithmetic of every kernel that has a choice (mvr_set_math).

    f32eq   : every fp32 product on the 3-term bf16 split (h + m + l, 6 MFMA products: fp32-equivalent operands).
    split16 : the 2-term fp16 split (h + l, 3 products, 22-bit operands) where a kernel has it, with the
              split-bf16 re-run of any launch whose operands leave the fp16 window.
    Returns {"mode", "dtype", "knobs"}: dtype derived from the mode as read back, never from `mode`."""
    L = lib()
    L.mvr_set_math({"f32eq": 0, "split16": 1}[mode])
    m = math_state()
    dtype = "f32 (bf16x3 MFMA operands)" if not m else "mixed: split-fp16 (22-bit) operands in " + MATH_KERNELS
    return {"mode": "split16" if m else "f32eq", "dtype": dtype, "knobs": {"split16": m}}


class force:
    """with force("generic_gemm"): ... — a fallback path forced for the block (mvr_debug_force; tests only)"""

    def __init__(self, what, value=1):
        self.what, self.value = FORCE[what], int(value)

    def __enter__(self):
        self.prev = lib().mvr_debug_force(self.what, self.value)
        return self

    def __exit__(self, *a):
        lib().mvr_debug_force(self.what, self.prev)


_ws_cache = {}
_flag_cache = {}


def flag_word(device=None):
    """A device int32 per (device, current stream): the range flag of the split-fp16 launches that take one
    (mvr_spconv).  Stream-ordered use: the call clears it before its split-fp16 pass."""
    idx = (device.index if device is not None and device.index is not None else torch.cuda.current_device())
    key = (idx, torch.cuda.current_stream(idx).cuda_stream)
    buf = _flag_cache.get(key)
    if buf is None:
        buf = torch.zeros(64, dtype=torch.int32, device=torch.device("cuda", idx))
        _flag_cache[key] = buf
    return buf


def workspace(nbytes, device):
    """Reusable scratch buffer per (device, current stream), grown on demand: launches on one stream are
    ordered, so consecutive calls can share it; a second stream gets its own."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (idx, torch.cuda.current_stream(idx).cuda_stream)
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)
        _ws_cache[key] = buf
    if _WS_POISON:   # debugging: 0x7f bytes (3.4e38) in every handed-out workspace (finds reads before writes)
        buf[:int(nbytes)].fill_(0x7F)
    return buf


_WS_POISON = os.environ.get("MVR_WS_POISON") == "1"
