"""Sparse convolution kernels (csrc/spconv.hip, the MinkowskiConvolution forward of
lib/descriptor/fcgf.py:118-227) against an fp64 gather-GEMM restatement: both split arithmetics on the
pre-split weight images (split-bf16, the default, and the opt-in split-fp16), every channel shape FCGF uses, partial stencils (-1 neighbours), the row order of mvr_kernel_map_order, the identity map (1x1x1 conv)
and the fused bias / BatchNorm / residual / ReLU epilogue; features outside the split-fp16 window re-run the
launch in split-bf16 (bit-identical results)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[1, 0], ids=["sp_fp16x2", "sp_bf16x3"])
def smath(request):
    from lib import _native as NV
    prev = NV.lib().mvr_set_spconv_math(request.param)
    yield request.param
    NV.lib().mvr_set_spconv_math(prev)


def _run(gpu, Cin, Cout, K, Mout, Min, perm=False, epi=True, seed=0, edit=None, raw=False, inplace=False):
    import torch
    from lib import _native as NV
    rng = np.random.default_rng(seed)
    feat = rng.standard_normal((Min, Cin)).astype(np.float32)
    if edit:
        edit(feat)
    if K == 1:
        nbr = None
        Mout = Min
    else:
        nbr = rng.integers(0, Min, size=(Mout, K)).astype(np.int32)
        nbr[rng.random((Mout, K)) < 0.5] = -1   # partial stencils
        nbr[rng.random(Mout) < 0.05] = -1       # a few rows with no neighbour at all
    W = (rng.standard_normal((K, Cin, Cout)) / np.sqrt(K * Cin)).astype(np.float32)
    bias = rng.standard_normal(Cout).astype(np.float32) if epi else None
    g, b = rng.random(Cout).astype(np.float32) + 0.5, rng.standard_normal(Cout).astype(np.float32)
    m, v = rng.standard_normal(Cout).astype(np.float32), rng.random(Cout).astype(np.float32) + 0.5
    res = rng.standard_normal((Mout, Cout)).astype(np.float32) if epi else None
    # fp64 reference
    ref = np.zeros((Mout, Cout))
    nb = np.arange(Min)[:, None] if nbr is None else nbr
    for k in range(nb.shape[1]):
        ok = nb[:, k] >= 0
        ref[ok] += feat[nb[ok, k]].astype(np.float64) @ W[k].astype(np.float64)
    if epi:
        ref = ((ref + bias - m) / np.sqrt(v.astype(np.float64) + 1e-5) * g + b) + res
        ref = np.maximum(ref, 0)
    d = lambda x: torch.from_numpy(x).to(gpu) if x is not None else None
    F, Wt, nbr_t, bias_t, res_t = d(feat), d(W), d(nbr), d(bias), d(res)
    gb, bb, mb, vb = d(g), d(b), d(m), d(v)
    L = NV.lib()
    perm_t = None
    if perm and nbr is not None:
        ws = torch.empty(L.mvr_kernel_map_order_bytes(Mout), dtype=torch.uint8, device=gpu)
        perm_t = torch.empty(Mout, dtype=torch.int32, device=gpu)
        NV.check(L.mvr_kernel_map_order(NV.ptr(nbr_t), None, 1, Mout, K, NV.ptr(perm_t), NV.ptr(ws), ws.numel(),
                                         NV.stream()),
                 "order")
    nbytes = L.mvr_spconv_wimage_bytes(K, Cin, Cout)
    wimg = torch.empty(nbytes, dtype=torch.uint8, device=gpu)
    NV.check(L.mvr_spconv_wimage(NV.ptr(Wt), K, Cin, Cout, NV.ptr(wimg), nbytes, NV.stream()), "wimage")
    out = res_t.clone() if inplace else torch.full((Mout, Cout), float("nan"), device=gpu)
    if inplace:
        res_t = out
    bn = NV.BnP(gb.data_ptr(), bb.data_ptr(), mb.data_ptr(), vb.data_ptr()) if epi else NV.BnP(None, None, None, None)
    rc = L.mvr_spconv(NV.ptr(F), Cin, Cin, NV.ptr(nbr_t), NV.ptr(perm_t), K, Mout, NV.ptr(Wt), Cout, NV.ptr(bias_t), bn,
                      1e-5, NV.ptr(res_t), Cout, int(epi), NV.ptr(out), Cout, NV.ptr(wimg),
                      NV.ptr(NV.flag_word(gpu)), NV.stream())
    assert rc == 0
    got = out.cpu().numpy()
    if raw:
        return got
    scale = np.abs(ref).max() + 1e-30
    err = np.abs(got - ref).max() / scale
    assert np.isfinite(got).all() and err < 2e-6, (Cin, Cout, K, err)


@pytest.mark.parametrize("cin,cout", [(32, 32), (32, 64), (64, 64), (64, 128), (128, 128), (128, 256), (256, 256),
                                      (256, 128), (256, 64), (128, 64), (96, 64)])
def test_spconv_3x3x3(gpu, cin, cout, smath):
    _run(gpu, cin, cout, 27, 1000, 900, perm=True, seed=cin + cout)


@pytest.mark.parametrize("cin,cout,mout", [(96, 64, 777), (64, 32, 300), (32, 32, 129)])
def test_spconv_identity_map(gpu, cin, cout, mout, smath):
    """1x1x1 convs (conv1_tr, final: fcgf.py:209-227) run with the identity map (nbr NULL)"""
    _run(gpu, cin, cout, 1, mout, mout, epi=cout != 32, seed=cin)


def test_spconv_ragged_rows_no_perm(gpu, smath):
    """a row count far from the tile size, natural row order, no epilogue, 8 offsets (transposed-conv size)"""
    _run(gpu, 64, 64, 8, 130, 2000, perm=False, epi=False, seed=9)


def test_spconv_requires_weight_image(gpu):
    """the exact-fp32 kernel of round 2 is gone: a call without the pre-split image is refused"""
    import torch
    from lib import _native as NV
    x = torch.zeros(8, 32, device=gpu)
    W = torch.zeros(1, 32, 32, device=gpu)
    rc = NV.lib().mvr_spconv(NV.ptr(x), 32, 32, None, None, 1, 8, NV.ptr(W), 32, None, NV.BnP(None, None, None, None),
                             1e-5, None, 0, 0, NV.ptr(x), 32, None, None, NV.stream())
    assert rc == -1


def test_spconv_rejects_channel_tail(gpu):
    """input channels come in whole 32-channel steps (an absent neighbour gathers a zero vector instead of masking
    each value): Cin % 32 != 0 is refused"""
    import torch
    from lib import _native as NV
    L = NV.lib()
    x = torch.zeros(8, 36, device=gpu)
    W = torch.zeros(1, 36, 32, device=gpu)
    nb = int(L.mvr_spconv_wimage_bytes(1, 36, 32))
    wimg = torch.zeros(nb, dtype=torch.uint8, device=gpu)
    rc = L.mvr_spconv(NV.ptr(x), 36, 36, None, None, 1, 8, NV.ptr(W), 32, None, NV.BnP(None, None, None, None),
                      1e-5, None, 0, 0, NV.ptr(x), 32, NV.ptr(wimg), None, NV.stream())
    assert rc == -1


def _big_feat(f):
    f[17, 5] = 2.0e3      # x 2^6 past 65504


def _tiny_feat(f):
    f *= 1.0e-6           # all below 2^-9


@pytest.mark.parametrize("edit,inplace", [(_big_feat, False), (_tiny_feat, False), (_big_feat, True), (None, True)])
def test_spconv_fp16_window(gpu, edit, inplace):
    """features outside the split-fp16 window re-run the launch in split-bf16; an output written over its residual
    runs split-bf16 directly: either way bit-identical to a split-bf16 launch (and within the fp64 tolerance)"""
    from lib import _native as NV
    L = NV.lib()
    outs = []
    prev = L.mvr_set_spconv_math(0)
    try:
        for m in (0, 1):
            L.mvr_set_spconv_math(m)
            outs.append(_run(gpu, 64, 128, 27, 1000, 900, perm=True, seed=4, edit=edit, raw=True, inplace=inplace))
        _run(gpu, 64, 128, 27, 1000, 900, perm=True, seed=4, edit=edit, inplace=inplace)
    finally:
        L.mvr_set_spconv_math(prev)
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("cin,cout", [(64, 128), (128, 256), (256, 128)])
def test_spconv_narrow_tiles_bit_identical(gpu, cin, cout, smath):
    """mvr_set_spconv_narrow: a small level's convs with more than 64 output channels on 64-channel column tiles
    (twice the workgroups) — each output column's reduction runs in the same order, so the bits do not change"""
    from lib import _native as NV
    L = NV.lib()
    prev = L.mvr_set_spconv_narrow(0)
    try:
        wide = _run(gpu, cin, cout, 27, 1000, 900, perm=True, seed=cin + cout, raw=True)
        L.mvr_set_spconv_narrow(1 << 30)
        narrow = _run(gpu, cin, cout, 27, 1000, 900, perm=True, seed=cin + cout, raw=True)
    finally:
        L.mvr_set_spconv_narrow(prev)
    assert np.array_equal(wide, narrow)
