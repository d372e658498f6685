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
    prev = NV.lib().mvr_set_math(request.param)
    yield request.param
    NV.lib().mvr_set_math(prev)


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


@pytest.mark.parametrize("planes", [False, True])
def test_spconv_transposed_map_more_outputs_than_inputs(gpu, planes, smath):
    """the shape of the round-4 spA1 fault: a transposed conv (up:4:256:128, fcgf.py:185-203) whose
    output set is ~4x its input set — the first FCGF layer where an output row index can exceed every input row —
    on a REAL kernel map (2 synthetic fragments, levels 8 -> 4), the ragged last 128-row tile, plus rows whose
    every neighbour is absent; fp64 reference.  The shipped kernel gathers only nbr[o][k] (input rows) and the zero
    vector for absent ones, so no output index is ever used as an input row."""
    import torch
    from lib import _native as NV
    from lib.sparse import voxelize, CoordinateManager
    from synth import synth_scene_fragments
    frags, _ = synth_scene_fragments(2, seed=12, n_pts=60000)
    c, _, counts, _ = voxelize(frags, 0.025, gpu)
    cm = CoordinateManager(c, len(counts))
    nbr = cm.kernel_map("up", 4).clone()
    Mout, Min = nbr.shape[0], cm.coords_at(8).shape[0]
    assert Mout > 3 * Min and Mout % 128 != 0
    nbr[5] = -1
    nbr[Mout - 1] = -1                                   # the ragged last tile's last row: no neighbour at all
    perm = cm.kernel_map_order("up", 4)
    rng = np.random.default_rng(3)
    cin, cout = 256, 128
    x = torch.from_numpy(np.maximum(rng.standard_normal((Min, cin)), 0).astype(np.float32)).to(gpu)
    W = torch.from_numpy((rng.standard_normal((27, cin, cout)) / np.sqrt(27 * cin)).astype(np.float32)).to(gpu)
    L = NV.lib()
    nb = L.mvr_spconv_wimage_bytes(27, cin, cout)
    wimg = torch.empty(nb, dtype=torch.uint8, device=gpu)
    NV.check(L.mvr_spconv_wimage(NV.ptr(W), 27, cin, cout, NV.ptr(wimg), nb, NV.stream()), "wimage")
    out = torch.full((Mout, cout), float("nan"), device=gpu)
    xp = _torch_planes(x) if planes else None
    NV.check(L.mvr_spconv_x(NV.ptr(x), cin, cin, NV.ptr(nbr), NV.ptr(perm), 27, Mout, NV.ptr(W), cout, None,
                            NV.BnP(None, None, None, None), 1e-5, None, 0, 0, NV.ptr(out), cout, NV.ptr(wimg),
                            NV.ptr(NV.flag_word(gpu)), NV.ptr(xp), None, NV.stream()), "mvr_spconv_x")
    got = out.cpu().numpy()
    nbn, xn, Wn = nbr.cpu().numpy(), x.cpu().numpy().astype(np.float64), W.cpu().numpy().astype(np.float64)
    ref = np.zeros((Mout, cout))
    for k in range(27):
        ok = nbn[:, k] >= 0
        ref[ok] += xn[nbn[ok, k]] @ Wn[k]
    assert np.isfinite(got).all()
    assert np.abs(got - ref).max() / np.abs(ref).max() < 2e-6
    assert (got[5] == 0).all() and (got[Mout - 1] == 0).all()


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
    prev = L.mvr_set_math(0)
    try:
        for m in (0, 1):
            L.mvr_set_math(m)
            outs.append(_run(gpu, 64, 128, 27, 1000, 900, perm=True, seed=4, edit=edit, raw=True, inplace=inplace))
        _run(gpu, 64, 128, 27, 1000, 900, perm=True, seed=4, edit=edit, inplace=inplace)
    finally:
        L.mvr_set_math(prev)
    assert np.array_equal(outs[0], outs[1])


def _torch_planes(x):
    """[M, C] fp32 -> [M, 3, C] int16: the RNE bf16 split h, m, l (x - h and r - m exact) — the split the sparse
    conv kernel applies to fp32 gathers (mfma_bf16.hpp split_pair<0>)"""
    import torch
    h = x.to(torch.bfloat16)
    r = x - h.float()
    m = r.to(torch.bfloat16)
    lo = (r - m.float()).to(torch.bfloat16)
    return torch.stack([h, m, lo], 1).view(torch.int16).contiguous()


@pytest.mark.parametrize("cin,cout,K,ld_off", [(32, 32, 27, 0), (64, 64, 27, 0), (128, 128, 27, 0), (256, 256, 27, 0),
                                               (256, 64, 27, 0), (96, 64, 1, 0), (64, 32, 1, 0), (32, 64, 27, 64)])
def test_spconv_presplit_planes_bit_identical(gpu, cin, cout, K, ld_off, smath):
    """mvr_spconv_x: gathering the input's pre-split bf16 planes (in_planes) gives the fp32-gather result bit for bit
    (the same split, done by the producer instead of at each of a row's gathers), also under split16 (its guarded
    split-bf16 re-run gathers the planes); the planes the call writes for its output (out_planes) equal the split of
    its fp32 output; the input may be a column slice of a wider buffer (ld_off: a concatenation's second half),
    ragged last tile, rows with no neighbour"""
    import torch
    from lib import _native as NV
    rng = np.random.default_rng(cin + cout + K)
    Min, Mout = 3001, 2777 if K > 1 else 3001
    ld = cin + ld_off
    wide = torch.from_numpy(np.maximum(rng.standard_normal((Min, ld)), 0).astype(np.float32)).to(gpu)
    x = wide[:, ld_off:]
    xp_all = _torch_planes(wide)
    xp = xp_all[:, :, ld_off:]
    nbr = None
    if K > 1:
        nb = rng.integers(0, Min, size=(Mout, K)).astype(np.int32)
        nb[rng.random((Mout, K)) < 0.6] = -1
        nb[rng.random(Mout) < 0.05] = -1
        nbr = torch.from_numpy(nb).to(gpu)
    W = torch.from_numpy((rng.standard_normal((K, cin, cout)) / np.sqrt(K * cin)).astype(np.float32)).to(gpu)
    L = NV.lib()
    nbytes = L.mvr_spconv_wimage_bytes(K, cin, cout)
    wimg = torch.empty(nbytes, dtype=torch.uint8, device=gpu)
    NV.check(L.mvr_spconv_wimage(NV.ptr(W), K, cin, cout, NV.ptr(wimg), nbytes, NV.stream()), "wimage")
    g = torch.rand(cout, device=gpu) + 0.5
    b, m, v = torch.randn(cout, device=gpu), torch.randn(cout, device=gpu), torch.rand(cout, device=gpu) + 0.5
    bn = NV.BnP(g.data_ptr(), b.data_ptr(), m.data_ptr(), v.data_ptr())
    outs = []
    for planes in (False, True):
        out = torch.full((Mout, cout), float("nan"), device=gpu)
        op = torch.zeros(Mout, 3, cout, dtype=torch.int16, device=gpu) if planes else None
        NV.check(L.mvr_spconv_x(NV.ptr(x), ld, cin, NV.ptr(nbr), None, K, Mout, NV.ptr(W), cout, None, bn, 1e-5,
                                None, 0, 1, NV.ptr(out), cout, NV.ptr(wimg), NV.ptr(NV.flag_word(gpu)),
                                NV.ptr(xp) if planes else None, NV.ptr(op), NV.stream()), "mvr_spconv_x")
        outs.append((out, op))
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0][0]).all()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[1][1], _torch_planes(outs[1][0]))
    # argument checks: misaligned planes / ld not a multiple of 8
    assert L.mvr_spconv_x(NV.ptr(x), ld, cin, NV.ptr(nbr), None, K, Mout, NV.ptr(W), cout, None, bn, 1e-5, None, 0, 1,
                          NV.ptr(outs[0][0]), cout, NV.ptr(wimg), None, xp.data_ptr() + 2, None, NV.stream()) != 0


def test_fcgf_presplit_equals_fp32_gathers(gpu, monkeypatch):
    """FCGFNet end to end with every conv's planes (the default) equals the fp32-gather path bit for bit"""
    import torch
    import lib.descriptor.fcgf as fc
    from synth import synth_scene_fragments, synth_state
    from lib.sparse import voxelize, SparseTensor
    frags, _ = synth_scene_fragments(2, seed=6, n_pts=60000)
    net = fc.FCGFNet()
    st = synth_state({k: tuple(v.shape) for k, v in net.state_dict().items()}, seed=8)
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    net = net.to(gpu).eval()
    c, _, _, _ = voxelize(frags, 0.025, gpu)
    F = torch.ones(c.shape[0], 1, device=gpu)
    outs = []
    for pre in (True, False):
        monkeypatch.setattr(fc, "PRESPLIT", pre)
        with torch.no_grad():
            outs.append(net(SparseTensor(F, coords=c).to(gpu)).F.clone())
    assert torch.equal(outs[0], outs[1])
