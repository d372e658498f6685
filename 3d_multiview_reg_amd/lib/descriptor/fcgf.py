"""FCGF fully-convolutional geometric features (reference lib/descriptor/fcgf.py)
on MI355X.

Same constructor and parameter tree as the reference's FCGFNet (MinkowskiEngine
0.4 naming: '<conv>.kernel' [K, Cin, Cout], '<norm>.bn.*' BatchNorm1d,
'final.bias'), so FCGF checkpoints load by key.  forward() runs the 4-level
sparse U-Net as ~30 native launches over ALL fragments of the batch at once:
voxel hash / strided coordinate sets / neighbour tables (cached on the
CoordinateManager) and the gather-GEMM sparse convolution with BatchNorm,
residual and ReLU fused into its epilogue; skip concatenations are free (the
producers write straight into the halves of the concatenated buffers).
"""
import os

import torch
import torch.nn as nn

from lib import _native as N
from lib.sparse import SparseTensor


# conv1 (7^3) as brick-tiled dense windows on split-bf16 MFMA (csrc/sparse.hip spconv_c1_brick_kernel);
# MVR_CONV1_BRICKS=0 selects the per-row gather kernel (A/B timing)
CONV1_BRICKS = os.environ.get("MVR_CONV1_BRICKS", "1") == "1"
# MVR_SPCONV_PRESPLIT=1: every conv's output also written as split-bf16 planes that the next conv gathers instead of
# re-splitting fp32 rows in its inner loop (csrc/spconv.hip PS = 1; bit-identical).  Off by default: measured slower
# on the same box (round 6, profiles/r06/ab_r6s1.txt: the sparse convs 6.63 ms per step with fp32 gathers vs 8.40 with
# the planes — 6 instead of 4 bytes per gathered value, and the level-1 planes no longer fit the Infinity Cache)
PRESPLIT = os.environ.get("MVR_SPCONV_PRESPLIT", "0") == "1"


def _planes(M, ld, dev):
    """[M, 3, ld] bf16 planes (h, m, l) of an [M, ld] fp32 activation buffer (views of it slice the last dim like
    the fp32 buffer's columns), or None without PRESPLIT"""
    return torch.empty(M, 3, ld, dtype=torch.int16, device=dev) if PRESPLIT else None


class _MEConv(nn.Module):
    """Parameter holder with MinkowskiConvolution(0.4)'s names."""

    def __init__(self, cin, cout, ksize, has_bias=False):
        super().__init__()
        self.kernel_size = ksize
        self.kernel = nn.Parameter(torch.empty(ksize ** 3, cin, cout))
        nn.init.kaiming_normal_(self.kernel.data.view(-1, cout), nonlinearity="relu")
        self.bias = nn.Parameter(torch.zeros(1, cout)) if has_bias else None
        self._wimg = None
        self._wimg_key = None

    def wimage(self):
        """Split-bf16 weight image (mvr_spconv_wimage), rebuilt when the kernel tensor changes."""
        k = self.kernel
        key = (k.data_ptr(), k._version, k.device)
        if self._wimg is None or self._wimg_key != key:
            K, cin, cout = k.shape
            nb = N.lib().mvr_spconv_wimage_bytes(K, cin, cout)
            self._wimg = torch.empty(nb, dtype=torch.uint8, device=k.device)
            N.check(N.lib().mvr_spconv_wimage(N.ptr(k.data), K, cin, cout, N.ptr(self._wimg), nb, N.stream()),
                    "mvr_spconv_wimage")
            self._wimg_key = key
        return self._wimg


class _MENorm(nn.Module):
    """MinkowskiBatchNorm: wraps BatchNorm1d as `.bn` (fcgf.py:14-20)."""

    def __init__(self, c, momentum=0.05):
        super().__init__()
        self.bn = nn.BatchNorm1d(c, momentum=momentum)


class BasicBlockBN(nn.Module):
    """fcgf.py:23-67: conv-bn-relu-conv-bn + residual, relu."""

    def __init__(self, inplanes, planes, bn_momentum=0.1):
        super().__init__()
        self.conv1 = _MEConv(inplanes, planes, 3)
        self.norm1 = _MENorm(planes, bn_momentum)
        self.conv2 = _MEConv(planes, planes, 3)
        self.norm2 = _MENorm(planes, bn_momentum)


def _bn(norm):
    if norm is None:
        return N.BnP(None, None, None, None), 1e-5
    b = norm.bn
    return N.BnP(b.weight.data_ptr(), b.bias.data_ptr(), b.running_mean.data_ptr(), b.running_var.data_ptr()), b.eps


class FCGFNet(nn.Module):
    NORM_TYPE = "BN"
    BLOCK_NORM_TYPE = "BN"
    CHANNELS = [None, 32, 64, 128, 256]
    TR_CHANNELS = [None, 64, 64, 64, 128]

    def __init__(self, in_channels=1, out_channels=32, bn_momentum=0.05, normalize_feature=True,
                 conv1_kernel_size=7, D=3):
        super().__init__()
        C, T = self.CHANNELS, self.TR_CHANNELS
        self.D = D
        self.normalize_feature = normalize_feature
        self.conv1_kernel_size = conv1_kernel_size
        self.conv1 = _MEConv(in_channels, C[1], conv1_kernel_size)
        self.norm1 = _MENorm(C[1], bn_momentum)
        self.block1 = BasicBlockBN(C[1], C[1], bn_momentum)
        self.conv2 = _MEConv(C[1], C[2], 3)
        self.norm2 = _MENorm(C[2], bn_momentum)
        self.block2 = BasicBlockBN(C[2], C[2], bn_momentum)
        self.conv3 = _MEConv(C[2], C[3], 3)
        self.norm3 = _MENorm(C[3], bn_momentum)
        self.block3 = BasicBlockBN(C[3], C[3], bn_momentum)
        self.conv4 = _MEConv(C[3], C[4], 3)
        self.norm4 = _MENorm(C[4], bn_momentum)
        self.block4 = BasicBlockBN(C[4], C[4], bn_momentum)
        self.conv4_tr = _MEConv(C[4], T[4], 3)
        self.norm4_tr = _MENorm(T[4], bn_momentum)
        self.block4_tr = BasicBlockBN(T[4], T[4], bn_momentum)
        self.conv3_tr = _MEConv(C[3] + T[4], T[3], 3)
        self.norm3_tr = _MENorm(T[3], bn_momentum)
        self.block3_tr = BasicBlockBN(T[3], T[3], bn_momentum)
        self.conv2_tr = _MEConv(C[2] + T[3], T[2], 3)
        self.norm2_tr = _MENorm(T[2], bn_momentum)
        self.block2_tr = BasicBlockBN(T[2], T[2], bn_momentum)
        self.conv1_tr = _MEConv(C[1] + T[2], T[1], 1)
        self.final = _MEConv(T[1], out_channels, 1, has_bias=True)

    # ------------------------------------------------------------------ native helpers
    def _conv(self, x, ldx, conv, km, M, out, ldout, norm=None, res=None, ldres=0, relu=False, bias=None, xp=None,
              outp=None):
        """km: (neighbour table, row order) of lib.sparse.CoordinateManager, or None for a 1x1x1 conv.  xp / outp:
        the split-bf16 planes of x (gathered instead of x) / of out (written beside it), or None."""
        bnp, eps = _bn(norm)
        K, cin, cout = conv.kernel.shape
        nbr, perm = km if km is not None else (None, None)
        # split-bf16 sparse convs (csrc/spconv.hip) on weights pre-split once per weight version
        wimg = conv.wimage()
        N.check(N.lib().mvr_spconv_x(N.ptr(x), ldx, cin, N.ptr(nbr), N.ptr(perm), K, M, N.ptr(conv.kernel), cout,
                                     N.ptr(bias), bnp, eps, N.ptr(res), ldres, int(relu), N.ptr(out), ldout,
                                     N.ptr(wimg), N.ptr(N.flag_word(x.device)), N.ptr(xp), N.ptr(outp), N.stream()),
                "mvr_spconv_x")
        return out

    def _block(self, blk, x, ldx, km, M, out, ldout, xp=None, outp=None):
        """BasicBlockBN at one stride; x may live inside a wider buffer (ldx)."""
        c = blk.conv1.kernel.shape[2]
        t = torch.empty(M, c, device=x.device)
        tp = _planes(M, c, x.device)
        self._conv(x, ldx, blk.conv1, km, M, t, c, blk.norm1, relu=True, xp=xp, outp=tp)
        self._conv(t, c, blk.conv2, km, M, out, ldout, blk.norm2, res=x, ldres=ldx, relu=True, xp=tp, outp=outp)
        return out

    def forward(self, x):
        N.require_hip()
        f32 = torch.float32
        if not all(t.is_cuda and t.dtype is f32 and t.is_contiguous()
                   for t in (*self.parameters(), *self.buffers()) if t.dtype.is_floating_point):
            raise RuntimeError("FCGFNet parameters must be contiguous float32 on a HIP device")
        if self.training:
            raise NotImplementedError("FCGFNet on the HIP path runs in eval mode (BatchNorm running statistics)")
        cm = x.coords_man
        cm.prepare_orders()   # all ten 3^3 maps and their row orders up front: one radix sort for the ten orders

        def km(kind, s):
            return cm.kernel_map(kind, s), cm.kernel_map_order(kind, s)
        dev = x.F.device
        C, T = self.CHANNELS, self.TR_CHANNELS
        M = [cm.coords_at(s).shape[0] for s in (1, 2, 4, 8)]
        L = N.lib()
        feat = x.F.float().contiguous()
        if feat.shape[1] != 1:
            raise NotImplementedError("conv1 kernel supports in_channels=1 (all reference configs)")
        # conv1 (7^3, 1 -> 32) + norm1
        s1 = torch.empty(M[0], C[1], device=dev)
        bnp, eps = _bn(self.norm1)
        bricks = cm.brick_map(1)
        # the output set is the input set: out_coords NULL selects the brick-tiled MFMA kernel (7^3 only)
        oc = None if (self.conv1_kernel_size == 7 and CONV1_BRICKS) else N.ptr(cm.coords_at(1))
        s1p = _planes(M[0], C[1], dev) if oc is None else None
        N.check(L.mvr_spconv_c1_x(oc, M[0], N.ptr(bricks), M[0], bricks.numel(), N.ptr(feat),
                                  self.conv1_kernel_size, 1, N.ptr(self.conv1.kernel), C[1], bnp, eps, 0, N.ptr(s1),
                                  C[1], N.ptr(s1p), N.stream()), "mvr_spconv_c1_x")
        # concatenation buffers: [tr-branch | skip] (and their planes, sliced the same way)
        cat1 = torch.empty(M[0], T[2] + C[1], device=dev)      # 64 + 32
        cat2 = torch.empty(M[1], T[3] + C[2], device=dev)      # 64 + 64
        cat3 = torch.empty(M[2], T[4] + C[3], device=dev)      # 128 + 128
        w1, w2, w3 = cat1.shape[1], cat2.shape[1], cat3.shape[1]
        cat1p, cat2p, cat3p = (_planes(M[i], w, dev) for i, w in ((0, w1), (1, w2), (2, w3)))
        skip1, skip2, skip3 = cat1[:, T[2]:], cat2[:, T[3]:], cat3[:, T[4]:]

        def sl(p, c0):   # the planes of the columns [c0, ...) of a concatenation buffer
            return p[:, :, c0:] if p is not None else None
        skip1p, skip2p, skip3p = sl(cat1p, T[2]), sl(cat2p, T[3]), sl(cat3p, T[4])
        # encoder
        self._block(self.block1, s1, C[1], km("s1", 1), M[0], skip1, w1, s1p, skip1p)   # out_s1 (relu'd)
        t2 = torch.empty(M[1], C[2], device=dev)
        t2p = _planes(M[1], C[2], dev)
        self._conv(skip1, w1, self.conv2, km("down", 1), M[1], t2, C[2], self.norm2, xp=skip1p, outp=t2p)
        self._block(self.block2, t2, C[2], km("s1", 2), M[1], skip2, w2, t2p, skip2p)    # out_s2
        t3 = torch.empty(M[2], C[3], device=dev)
        t3p = _planes(M[2], C[3], dev)
        self._conv(skip2, w2, self.conv3, km("down", 2), M[2], t3, C[3], self.norm3, xp=skip2p, outp=t3p)
        self._block(self.block3, t3, C[3], km("s1", 4), M[2], skip3, w3, t3p, skip3p)    # out_s4
        t4 = torch.empty(M[3], C[4], device=dev)
        t4p = _planes(M[3], C[4], dev)
        self._conv(skip3, w3, self.conv4, km("down", 4), M[3], t4, C[4], self.norm4, xp=skip3p, outp=t4p)
        s8 = torch.empty(M[3], C[4], device=dev)
        s8p = _planes(M[3], C[4], dev)
        self._block(self.block4, t4, C[4], km("s1", 8), M[3], s8, C[4], t4p, s8p)        # out_s8
        # decoder
        u = torch.empty(M[2], T[4], device=dev)
        up = _planes(M[2], T[4], dev)
        self._conv(s8, C[4], self.conv4_tr, km("up", 4), M[2], u, T[4], self.norm4_tr, xp=s8p, outp=up)
        self._block(self.block4_tr, u, T[4], km("s1", 4), M[2], cat3, w3, up, cat3p)     # out_s4_tr
        u = torch.empty(M[1], T[3], device=dev)
        up = _planes(M[1], T[3], dev)
        self._conv(cat3, w3, self.conv3_tr, km("up", 2), M[1], u, T[3], self.norm3_tr, xp=cat3p, outp=up)
        self._block(self.block3_tr, u, T[3], km("s1", 2), M[1], cat2, w2, up, cat2p)     # out_s2_tr
        u = torch.empty(M[0], T[2], device=dev)
        up = _planes(M[0], T[2], dev)
        self._conv(cat2, w2, self.conv2_tr, km("up", 1), M[0], u, T[2], self.norm2_tr, xp=cat2p, outp=up)
        self._block(self.block2_tr, u, T[2], km("s1", 1), M[0], cat1, w1, up, cat1p)     # out_s1_tr
        h = torch.empty(M[0], T[1], device=dev)
        hp = _planes(M[0], T[1], dev)
        self._conv(cat1, w1, self.conv1_tr, None, M[0], h, T[1], relu=True, xp=cat1p, outp=hp)
        cout = self.final.kernel.shape[2]
        out = torch.empty(M[0], cout, device=dev)
        self._conv(h, T[1], self.final, None, M[0], out, cout, bias=self.final.bias, xp=hp)
        if self.normalize_feature:
            N.check(L.mvr_l2norm_rows(N.ptr(out), M[0], cout, cout, N.stream()), "mvr_l2norm_rows")
        return SparseTensor(out, coords_key=1, coords_manager=cm)
