"""FCGF sparse-voxel descriptor restated in numpy (TEST ORACLE ONLY).

Restates lib/descriptor/fcgf.py:97-280 (FCGFNet.forward) on top of a numpy
re-statement of the MinkowskiEngine 0.4 primitives it calls.
MinkowskiEngine (github StanfordVL/MinkowskiEngine, unpinned — the reference
README clones master, README.md:56; API era v0.4.x) is NOT vendored in the
reference and cannot run here, so these conventions are OURS and the FCGF
parity is "unpinned" (DESIGN.md §Oracle):
  * quantisation: coords = floor(xyz / voxel) (float64), first occurrence kept,
    output in first-occurrence order (ME.utils.sparse_quantize(return_index=True));
  * strided coordinates floor(c / s) * s, first-occurrence order over the finer rows;
  * stencil offset index k = (dx+r) + ks*(dy+r) + ks^2*(dz+r), offsets scaled by the
    input tensor stride; transposed conv: input = output - off * s_out;
  * weights: conv '.kernel' [K, Cin, Cout] (ME 0.4), BatchNorm1d eval (eps 1e-5).
"""
import ctypes
import os

import numpy as np

KEY_BIAS = 1 << 16
_C = None


def _clib():
    """oracle/build/libmvoracle.so (oracle/csrc/sparse_conv.c, C + OpenMP: built by __graft_entry__.build() or
    `make -C oracle`): the kernel map and sparse conv of this module for the host-core CPU baseline"""
    global _C
    if _C is None:
        # MVO_LIB: another build of the same source (tests/test_oracle_sanitize.py: the ASan + UBSan build)
        path = os.environ.get("MVO_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "build",
                                                         "libmvoracle.so")
        L = ctypes.CDLL(path)
        vp, i64, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        L.mvo_kernel_map.argtypes = [vp, i64, vp, i64, ci, ci, ci, vp]
        L.mvo_sparse_conv.argtypes = [vp, i64, ci, vp, i64, ci, vp, ci, vp, vp]
        L.mvo_set_threads.argtypes = [ci]
        L.mvo_isa.argtypes = []
        _C = L
    return _C


def set_threads(n):
    """OpenMP threads of the C backend; returns the previous maximum"""
    return _clib().mvo_set_threads(int(n))


def isa():
    """'avx2+fma' when the C sparse conv runs its haswell clone on this host, else 'x86-64' (recorded with the CPU
    baseline)"""
    return "avx2+fma" if _clib().mvo_isa() else "x86-64"


def kernel_map_c(out_coords, in_coords, ks, step, transposed=False):
    """kernel_map() in C (hash of the input set instead of the sorted-key table): the same nbr"""
    oc = np.ascontiguousarray(out_coords, dtype=np.int32)
    ic = np.ascontiguousarray(in_coords, dtype=np.int32)
    nbr = np.empty((len(oc), ks ** 3), dtype=np.int64)
    rc = _clib().mvo_kernel_map(ic.ctypes.data, len(ic), oc.ctypes.data, len(oc), ks, step, int(transposed),
                                nbr.ctypes.data)
    if rc:
        raise RuntimeError("mvo_kernel_map failed (%d)" % rc)
    return nbr


def sparse_conv_c(feat, nbr, W, bias=None):
    """sparse_conv() in C + OpenMP (fp32, per output row in the order k, ci)"""
    f = np.ascontiguousarray(feat, dtype=np.float32)
    n = np.ascontiguousarray(nbr, dtype=np.int64)
    w = np.ascontiguousarray(W, dtype=np.float32)
    b = None if bias is None else np.ascontiguousarray(np.asarray(bias, np.float32).reshape(-1))
    out = np.empty((n.shape[0], w.shape[2]), dtype=np.float32)
    rc = _clib().mvo_sparse_conv(f.ctypes.data, f.shape[0], f.shape[1], n.ctypes.data, n.shape[0], n.shape[1],
                                 w.ctypes.data, w.shape[2], None if b is None else b.ctypes.data, out.ctypes.data)
    if rc:
        raise RuntimeError("mvo_sparse_conv failed (%d)" % rc)
    return out


def pack(c):
    """c int [M,4] (b, x, y, z) -> int64 keys (same packing as csrc/sparse.hip)."""
    c = np.asarray(c, dtype=np.int64)
    return ((c[:, 0] << 51) | (((c[:, 1] + KEY_BIAS) & 0x1FFFF) << 34) | (((c[:, 2] + KEY_BIAS) & 0x1FFFF) << 17)
            | ((c[:, 3] + KEY_BIAS) & 0x1FFFF))


def first_occurrence(keys):
    """indices of the first occurrence of every distinct key, in source order."""
    _, idx = np.unique(keys, return_index=True)
    return np.sort(idx)


def voxelize(xyz_list, voxel):
    """scripts/pairwise_demo.py:74-96 / scripts/utils.py:102-113.
    Returns coords int32 [M,4] (b,x,y,z), sel (global point index), per-fragment counts."""
    coords, sel, counts = [], [], []
    base = 0
    for b, xyz in enumerate(xyz_list):
        q = np.floor(np.asarray(xyz, dtype=np.float64) / voxel).astype(np.int64)
        c = np.concatenate([np.full((len(q), 1), b, np.int64), q], axis=1)
        keep = first_occurrence(pack(c))
        coords.append(c[keep])
        sel.append(keep + base)
        counts.append(len(keep))
        base += len(xyz)
    return np.concatenate(coords).astype(np.int32), np.concatenate(sel), np.asarray(counts)


def downsample(coords, s):
    c = np.asarray(coords, dtype=np.int64).copy()
    c[:, 1:] = np.floor_divide(c[:, 1:], s) * s
    keep = first_occurrence(pack(c))
    return c[keep].astype(np.int32)


class Table:
    def __init__(self, coords):
        k = pack(coords)
        self.order = np.argsort(k, kind="stable")
        self.sk = k[self.order]

    def find(self, coords):
        k = pack(coords)
        i = np.searchsorted(self.sk, k)
        i = np.minimum(i, len(self.sk) - 1)
        hit = self.sk[i] == k
        return np.where(hit, self.order[i], -1)


def offsets(ks):
    r = ks // 2
    k = np.arange(ks ** 3)
    return np.stack([k % ks - r, (k // ks) % ks - r, k // (ks * ks) - r], axis=1)


def kernel_map(out_coords, in_table, ks, step, transposed=False):
    """nbr [Mo, ks^3]: row of out + sign*off*step in the input set, -1 if absent."""
    oc = np.asarray(out_coords, dtype=np.int64)
    sign = -1 if transposed else 1
    nbr = np.empty((len(oc), ks ** 3), dtype=np.int64)
    for k, off in enumerate(offsets(ks)):
        q = oc.copy()
        q[:, 1:] += sign * off * step
        nbr[:, k] = in_table.find(q)
    return nbr


def sparse_conv(feat, nbr, W, bias=None):
    """out[o] = sum_k feat[nbr[o,k]] @ W[k]  (MinkowskiConvolution forward)."""
    out = np.zeros((nbr.shape[0], W.shape[2]), dtype=np.float32)
    for k in range(nbr.shape[1]):
        v = nbr[:, k] >= 0
        if v.any():
            out[v] += feat[nbr[v, k]] @ W[k]
    if bias is not None:
        out += np.asarray(bias, np.float32).reshape(1, -1)
    return out


def bn(x, st, pre, eps=1e-5):
    g, b = st[pre + ".bn.weight"], st[pre + ".bn.bias"]
    m, v = st[pre + ".bn.running_mean"], st[pre + ".bn.running_var"]
    return ((x - m) / np.sqrt(v + np.float32(eps)) * g + b).astype(np.float32)


def relu(x):
    return np.maximum(x, 0)


class Levels:
    """Coordinate sets, tables and kernel maps for strides 1, 2, 4, 8 of a batch (backend "c": the maps by
    oracle/csrc/sparse_conv.c)."""

    def __init__(self, coords0, backend="numpy"):
        self.coords = [np.asarray(coords0, np.int32)]
        for l in range(1, 4):
            self.coords.append(downsample(self.coords[-1], 2 ** l))
        self.backend = backend
        self.tables = [Table(c) for c in self.coords] if backend == "numpy" else None
        self._maps = {}

    def nbr(self, kind, l):
        key = (kind, l)
        if key not in self._maps:
            # (output level, input level, ks, step, transposed)
            o, i, ks, step, tr = {"s1": (l, l, 3, 2 ** l, False), "down": (l + 1, l, 3, 2 ** l, False),
                                  "up": (l, l + 1, 3, 2 ** l, True), "k7": (0, 0, 7, 1, False)}[kind]
            if self.backend == "c":
                m = kernel_map_c(self.coords[o], self.coords[i], ks, step, tr)
            else:
                m = kernel_map(self.coords[o], self.tables[i], ks, step, tr)
            self._maps[key] = m
        return self._maps[key]


def block(x, st, pre, lv, l, conv=None):
    """BasicBlockBN (fcgf.py:23-67): relu(bn1(conv1 x)) -> bn2(conv2) + x -> relu."""
    conv = conv or sparse_conv
    n = lv.nbr("s1", l)
    o = relu(bn(conv(x, n, st[pre + ".conv1.kernel"]), st, pre + ".norm1"))
    o = bn(conv(o, n, st[pre + ".conv2.kernel"]), st, pre + ".norm2")
    return relu(o + x)


def fcgf_forward(st, coords0, feats0, normalize=True, backend="numpy"):
    """fcgf.py:229-280 (eval).  st: state dict of numpy arrays (ME 0.4 key names).
    coords0 int [M,4], feats0 [M,1] -> F [M,32] (+ the Levels used).  backend "c": kernel maps and sparse convs
    in C + OpenMP (oracle/csrc/sparse_conv.c; the CPU baseline's FCGF leg), else numpy."""
    st = {k: np.asarray(v, np.float32) for k, v in st.items() if not k.endswith("num_batches_tracked")}
    lv = Levels(coords0, backend)
    sparse_conv = sparse_conv_c if backend == "c" else globals()["sparse_conv"]
    blk = lambda x, pre, l: block(x, st, pre, lv, l, sparse_conv)   # noqa: E731
    f = np.asarray(feats0, np.float32)
    s1 = bn(sparse_conv(f, lv.nbr("k7", 0), st["conv1.kernel"]), st, "norm1")
    s1 = blk(s1, "block1", 0)
    out = relu(s1)
    s2 = bn(sparse_conv(out, lv.nbr("down", 0), st["conv2.kernel"]), st, "norm2")
    s2 = blk(s2, "block2", 1)
    out = relu(s2)
    s4 = bn(sparse_conv(out, lv.nbr("down", 1), st["conv3.kernel"]), st, "norm3")
    s4 = blk(s4, "block3", 2)
    out = relu(s4)
    s8 = bn(sparse_conv(out, lv.nbr("down", 2), st["conv4.kernel"]), st, "norm4")
    s8 = blk(s8, "block4", 3)
    out = relu(s8)
    out = bn(sparse_conv(out, lv.nbr("up", 2), st["conv4_tr.kernel"]), st, "norm4_tr")
    out = relu(blk(out, "block4_tr", 2))
    out = np.concatenate([out, s4], axis=1)
    out = bn(sparse_conv(out, lv.nbr("up", 1), st["conv3_tr.kernel"]), st, "norm3_tr")
    out = relu(blk(out, "block3_tr", 1))
    out = np.concatenate([out, s2], axis=1)
    out = bn(sparse_conv(out, lv.nbr("up", 0), st["conv2_tr.kernel"]), st, "norm2_tr")
    out = relu(blk(out, "block2_tr", 0))
    out = np.concatenate([out, s1], axis=1)
    out = relu(out @ st["conv1_tr.kernel"][0])
    out = out @ st["final.kernel"][0] + st["final.bias"].reshape(1, -1)
    if normalize:
        out = out / np.linalg.norm(out, axis=1, keepdims=True)
    return out.astype(np.float32), lv


FCGF_CHANNELS = [None, 32, 64, 128, 256]
FCGF_TR_CHANNELS = [None, 64, 64, 64, 128]


def fcgf_state_shapes(in_channels=1, out_channels=32, conv1_kernel_size=7):
    """ME 0.4 state-dict key -> shape for FCGFNet (fcgf.py:105-227)."""
    C, T = FCGF_CHANNELS, FCGF_TR_CHANNELS
    sh = {}

    def conv(name, k, cin, cout):
        sh[name + ".kernel"] = (k ** 3, cin, cout)

    def norm(name, c):
        for s in ("weight", "bias", "running_mean", "running_var"):
            sh["%s.bn.%s" % (name, s)] = (c,)
        sh[name + ".bn.num_batches_tracked"] = ()

    def blk(name, c):
        conv(name + ".conv1", 3, c, c)
        norm(name + ".norm1", c)
        conv(name + ".conv2", 3, c, c)
        norm(name + ".norm2", c)

    conv("conv1", conv1_kernel_size, in_channels, C[1]); norm("norm1", C[1]); blk("block1", C[1])
    conv("conv2", 3, C[1], C[2]); norm("norm2", C[2]); blk("block2", C[2])
    conv("conv3", 3, C[2], C[3]); norm("norm3", C[3]); blk("block3", C[3])
    conv("conv4", 3, C[3], C[4]); norm("norm4", C[4]); blk("block4", C[4])
    conv("conv4_tr", 3, C[4], T[4]); norm("norm4_tr", T[4]); blk("block4_tr", T[4])
    conv("conv3_tr", 3, C[3] + T[4], T[3]); norm("norm3_tr", T[3]); blk("block3_tr", T[3])
    conv("conv2_tr", 3, C[2] + T[3], T[2]); norm("norm2_tr", T[2]); blk("block2_tr", T[2])
    conv("conv1_tr", 1, C[1] + T[2], T[1])
    conv("final", 1, T[1], out_channels)
    sh["final.bias"] = (1, out_channels)
    return sh
