"""Fused split-bf16 (fp32-equivalent) MFMA GEMM (csrc/gemm.hip) vs a float64 numpy reference, every
prologue/epilogue combination the OANet schedule uses, ragged shapes, padded rows."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BT = 128  # GEMM tile (csrc/gemm.hpp)


def r4(x):
    return (x + 3) // 4 * 4


def _pad(a, width):
    out = np.zeros(a.shape[:-1] + (width,), a.dtype)
    out[..., :a.shape[-1]] = a
    return out


def _run(gpu, M, N, K, batch, pro, bkc, bias_mode, stats_mode, res, seed=0, shared_a=False, math=1, edit=None,
         raw=False):
    import torch
    from lib import _native as NV
    r = np.random.RandomState(seed)
    K4, N4 = r4(K), r4(N)
    A = r.standard_normal((1 if shared_a else batch, M, K)).astype(np.float32)
    Bm = r.standard_normal((batch, K, N)).astype(np.float32)       # logical B(k, n)
    if pro == 3:
        Bm = np.abs(Bm)
    if edit:
        edit(A, Bm)
    Bstore = _pad(np.swapaxes(Bm, 1, 2), K4) if bkc else _pad(Bm, N4)
    Rm = r.standard_normal((batch, M, N)).astype(np.float32) if res else None
    bias = r.standard_normal(M if bias_mode == 1 else N).astype(np.float32) if bias_mode else None
    sc = sh = fac = None
    KT = (K + BT - 1) // BT
    if pro in (1, 2):
        sc = r.uniform(0.5, 1.5, (batch, K)).astype(np.float32)
        sh = r.uniform(-0.5, 0.5, (batch, K)).astype(np.float32)
    elif pro == 3:
        fac = _pad(r.uniform(0.1, 1.5, (batch, KT, N)).astype(np.float32), N4)
    # reference in float64
    Ad, Bd = A.astype(np.float64), Bm.astype(np.float64)
    if pro == 1:
        Ad = np.maximum(Ad * sc[:, None, :] + sh[:, None, :], 0)
    elif pro == 2:
        Bd = np.maximum(Bd * sc[:, :, None] + sh[:, :, None], 0)
    elif pro == 3:
        Bd = Bd * np.repeat(fac[:, :, :N].astype(np.float64), BT, axis=1)[:, :K]
    Cref = Ad @ Bd
    if bias_mode == 1:
        Cref += bias[None, :, None]
    elif bias_mode == 2:
        Cref += bias[None, None, :]
    if res:
        Cref += Rm
    dev = gpu
    t = lambda x: None if x is None else torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    tA, tB, tR, tb = t(_pad(A, K4)), t(Bstore), t(None if Rm is None else _pad(Rm, N4)), t(bias)
    tsc, tsh, tf = t(sc), t(sh), t(fac)
    C = torch.full((batch, M, N4), float("nan"), device=dev)
    nT = (N + BT - 1) // BT
    mT = (M + BT - 1) // BT
    if stats_mode in (1, 2):
        st = torch.zeros(batch, nT, M, 2, device=dev)
        st_ld = M
    elif stats_mode in (3, 4):
        st = torch.zeros(batch, mT, N, 2, device=dev)
        st_ld = N
    else:
        st, st_ld = None, 0
    if pro in (1, 2):
        pv, sPb, pld = (tsc, tsh), K, 0
    elif pro == 3:
        pv, sPb, pld = (tf, None), KT * N4, N4
    else:
        pv, sPb, pld = (None, None), 0, 0
    L = NV.lib()
    rc = L.mvr_gemm_f32(M, N, K, batch, NV.ptr(tA), 0 if shared_a else M * K4, K4, NV.ptr(tB),
                        K * N4 if not bkc else N * K4, K4 if bkc else N4, bkc,
                        NV.ptr(C), M * N4, N4, NV.ptr(tR), M * N4, NV.ptr(tb), bias_mode, NV.ptr(pv[0]),
                        NV.ptr(pv[1]), sPb, pld, pro, NV.ptr(st), st_ld, 0, stats_mode, math, NV.ptr(NV.flag_word()), NV.stream())
    assert rc == 0
    torch.cuda.synchronize()
    if raw:
        return C.cpu().numpy(), None if st is None else st.cpu().numpy()
    Cg = C.cpu().numpy().astype(np.float64)
    assert np.all(np.isfinite(Cg)), "padding columns must be written with finite values"
    Cg = Cg[..., :N]
    scale = np.abs(Ad) @ np.abs(Bd) + 1.0
    S = None if st is None else st.cpu().numpy().astype(np.float64)
    if stats_mode in (2, 3):
        # softmax epilogues store exp(v - tile max) and emit (tile max, sum)
        ax = -1 if stats_mode == 2 else 1
        nt = nT if stats_mode == 2 else mT
        for tt in range(nt):
            sl = (slice(None), slice(None), slice(tt * BT, (tt + 1) * BT)) if stats_mode == 2 else \
                (slice(None), slice(tt * BT, (tt + 1) * BT), slice(None))
            blk = Cref[sl]
            mx = blk.max(ax, keepdims=True)
            E = np.exp(blk - mx)
            # |d exp(v - m)| <= E * (|dv| + |dm|)
            tol = E * 4e-5 * scale[sl].max(ax, keepdims=True) + 1e-6
            assert np.all(np.abs(Cg[sl] - E) <= tol), np.max(np.abs(Cg[sl] - E) - tol)
            np.testing.assert_allclose(S[:, tt, :, 0], mx.squeeze(ax), rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(S[:, tt, :, 1], E.sum(ax), rtol=1e-4)
        return
    assert np.all(np.abs(Cg - Cref) <= 1e-5 * scale), np.max(np.abs(Cg - Cref) / scale)
    if S is None:
        return
    if stats_mode == 1:
        for tt in range(nT):
            blk = Cref[:, :, tt * BT:(tt + 1) * BT]
            np.testing.assert_allclose(S[:, tt, :, 0], blk.sum(-1), rtol=1e-4, atol=1e-3)
            dev2 = ((blk - blk.mean(-1, keepdims=True)) ** 2).sum(-1)      # squared deviations
            np.testing.assert_allclose(S[:, tt, :, 1], dev2, rtol=1e-4, atol=1e-3)
    else:
        for tt in range(mT):
            blk = Cref[:, tt * BT:(tt + 1) * BT, :]
            np.testing.assert_allclose(S[:, tt, :, 0], blk.sum(1), rtol=1e-4, atol=1e-3)
            dev2 = ((blk - blk.mean(1, keepdims=True)) ** 2).sum(1)
            np.testing.assert_allclose(S[:, tt, :, 1], dev2, rtol=1e-4, atol=1e-3)


# (pro, bkc, bias, stats, res) — the dispatch table of csrc/gemm.hip
COMBOS = [(0, 0, 1, 1, 0), (0, 0, 1, 0, 0), (2, 0, 1, 1, 0), (2, 0, 1, 0, 0), (2, 0, 1, 4, 0), (2, 0, 1, 1, 1),
          (2, 0, 1, 2, 0), (2, 0, 1, 3, 0), (3, 1, 0, 1, 0), (3, 0, 0, 1, 0), (1, 1, 2, 1, 1), (0, 0, 0, 0, 0),
          (0, 1, 0, 0, 0)]


@pytest.fixture(params=[1, 0], ids=["g_fp16x2", "g_bf16x3"])
def gf16(request):
    """mvr_set_math: split-math launches run split-fp16 first (guarded split-bf16 re-run) or split-bf16 only"""
    from lib import _native as NV
    prev = NV.lib().mvr_set_math(request.param)
    yield request.param
    NV.lib().mvr_set_math(prev)


@pytest.mark.parametrize("combo", COMBOS)
@pytest.mark.parametrize("shape", [(128, 256, 128, 2), (130, 517, 36, 3), (500, 300, 64, 1), (1, 40, 8, 2),
                                   (130, 518, 36, 3), (256, 1000, 500, 2), (128, 5000, 4, 1), (64, 999, 260, 2),
                                   (128, 5000, 128, 3), (128, 517, 128, 2), (128, 500, 128, 5), (128, 31, 128, 2),
                                   (128, 517, 256, 3), (128, 5000, 256, 2)])
def test_gemm_modes(gpu, combo, shape, gf16):
    """split arithmetic: split-fp16 first with its guarded split-bf16 re-run, or split-bf16 only (gf16)"""
    M, N, K, b = shape
    pro, bkc, bias, stats, res = combo
    if pro in (1, 2) and K % 4:
        pytest.skip("per-k prologue needs K % 4 == 0")
    _run(gpu, M, N, K, b, pro, bkc, bias, stats, res, seed=hash((combo, shape)) % 1000, shared_a=(pro != 1))


@pytest.mark.parametrize("shape", [(128, 32, 128, 1200), (128, 20, 128, 1100), (128, 33, 128, 1100)])
@pytest.mark.parametrize("combo", [(2, 0, 1, 1, 1), (2, 0, 1, 1, 0)])
def test_gemm_short_rows_many_pairs(gpu, combo, shape):
    """<= 1 point chunk per pair over > 1024 pairs: several pair changes per workgroup range (the point-conv
    kernel's per-pair fold staging; N <= 32 routes to the generic kernel)."""
    M, N, K, b = shape
    pro, bkc, bias, stats, res = combo
    _run(gpu, M, N, K, b, pro, bkc, bias, stats, res, seed=5, shared_a=True, math=1)


def test_gemm_ragged_k(gpu, gf16):
    # K = 6 (conv1 of reg_init, weight rows zero-padded to 8) and odd K for plain GEMMs
    _run(gpu, 128, 5000, 6, 2, 0, 0, 1, 1, 0, shared_a=True)
    _run(gpu, 128, 999, 7, 2, 0, 0, 1, 1, 0, shared_a=True)
    _run(gpu, 70, 333, 45, 2, 0, 1, 0, 0, 0)
    _run(gpu, 70, 333, 45, 2, 3, 1, 0, 1, 0)


def test_gemm_rejects_removed_math(gpu):
    """math must be 1 (split-bf16); the round-2 exact-fp32 value 0 is refused, not silently rerouted"""
    import torch
    from lib import _native as NV
    a = torch.zeros(128, 128, device=gpu)
    c = torch.empty(128, 128, device=gpu)
    rc = NV.lib().mvr_gemm_f32(128, 128, 128, 1, NV.ptr(a), 0, 128, NV.ptr(a), 0, 128, 0, NV.ptr(c), 0, 128, None, 0,
                               None, 0, None, None, 0, 0, 0, None, 0, 0, 0, 0, None, NV.stream())
    assert rc == -1


PCONV_COMBOS = [(2, 0, 1, 1, 0), (2, 0, 1, 1, 1), (2, 0, 1, 0, 0), (0, 0, 1, 0, 0), (0, 0, 1, 1, 0), (2, 0, 1, 0, 1)]


@pytest.fixture(params=[1, 0], ids=["pc_fp16x2", "pc_bf16x3"])
def pmath(request):
    from lib import _native as NV
    prev = NV.lib().mvr_set_math(request.param)
    yield request.param
    NV.lib().mvr_set_math(prev)


@pytest.mark.parametrize("combo", PCONV_COMBOS)
@pytest.mark.parametrize("shape", [(128, 5000, 128, 3), (128, 517, 256, 3), (128, 5000, 256, 2), (128, 500, 128, 5),
                                   (128, 33, 128, 1100)])
def test_pconv_maths(gpu, combo, shape, pmath):
    """the point-conv shapes (csrc/pconv.hip) on split-fp16 (weight rows range-scaled, activations x 2^6 after
    the prologue) and split-bf16: both within 1e-5 of the float64 result at its |A| |B| scale"""
    M, N, K, b = shape
    pro, bkc, bias, stats, res = combo
    if K == 256 and res:
        pytest.skip("the 256-channel convs have no residual form")
    _run(gpu, M, N, K, b, pro, bkc, bias, stats, res, seed=hash((combo, shape)) % 1000, shared_a=True, math=1)


def _big_b(A, B):
    B[1, 5, 7] = 7.0e4      # an activation past the fp16 range


def _big_b_pro(A, B):
    B[0, 9, 100] = 4.0e3    # ... past it after the prologue's x 2^6 (and sc <= 1.5)


def _tiny_b(A, B):
    B *= 1.0e-5             # raw activations all below 2^-9: re-run (the prologue lifts them: not there)


def _big_a(A, B):
    A *= 3.0e5              # weights: row-scaled, no re-run


@pytest.mark.parametrize("edit", [_big_b, _big_b_pro, _tiny_b, _big_a])
@pytest.mark.parametrize("combo", [(2, 0, 1, 1, 0), (0, 0, 1, 0, 0), (2, 0, 1, 1, 1)])
@pytest.mark.parametrize("K", [128, 256])
def test_pconv_fp16_range(gpu, edit, combo, K):
    """an activation outside the split-fp16 window re-runs the launch in split-bf16: outputs and statistics
    bit-identical to a split-bf16 launch; weights far past the fp16 range are scaled, not re-run"""
    from lib import _native as NV
    pro, bkc, bias, stats, res = combo
    if K == 256 and res:
        pytest.skip("the 256-channel convs have no residual form")
    if (edit is _big_b_pro and not pro) or (edit is _tiny_b and pro):
        pytest.skip("prologue case")
    L = NV.lib()
    outs = []
    prev = L.mvr_set_math(0)
    try:
        for m in (0, 1):
            L.mvr_set_math(m)
            outs.append(_run(gpu, 128, 700, K, 3, pro, bkc, bias, stats, res, seed=7, shared_a=True, edit=edit,
                             raw=True))
        if edit is not _big_a:   # (outputs ~1e8 there: the statistics' cancellation exceeds their fp64 tolerance)
            _run(gpu, 128, 700, K, 3, pro, bkc, bias, stats, res, seed=7, shared_a=True, edit=edit)   # vs float64
    finally:
        L.mvr_set_math(prev)
    (c0, s0), (c1, s1) = outs
    if edit is _big_a:
        assert not np.array_equal(c0, c1)
        np.testing.assert_allclose(c1, c0, rtol=1e-5, atol=1e-5 * np.abs(c0).max())
    else:
        assert np.array_equal(c0, c1, equal_nan=True)
        assert s0 is None or np.array_equal(s0, s1)


def test_pconv_in_place_residual(gpu):
    """out = conv(x) + out in place (the OANet PointCN / OAFilter form): the launch cannot be re-run once it has
    overwritten its residual, so it runs split-bf16 directly — with an out-of-range activation too, the result
    is the split-bf16 one bit for bit"""
    import torch
    from lib import _native as NV
    r = np.random.RandomState(11)
    P, M, N, K = 3, 128, 700, 128
    N4 = r4(N)
    A = (0.1 * r.standard_normal((M, K))).astype(np.float32)
    B = _pad(r.standard_normal((P, K, N)).astype(np.float32), N4)
    B[1, 3, 9] = 8.0e4
    R = _pad(r.standard_normal((P, M, N)).astype(np.float32), N4)
    bias = r.standard_normal(M).astype(np.float32)
    L = NV.lib()
    outs = []
    prev = L.mvr_set_math(0)
    try:
        for m in (0, 1):
            L.mvr_set_math(m)
            tA, tB, tb = (torch.from_numpy(x).to(gpu) for x in (A, B, bias))
            C = torch.from_numpy(R.copy()).to(gpu)
            assert L.mvr_gemm_f32(M, N, K, P, NV.ptr(tA), 0, K, NV.ptr(tB), K * N4, N4, 0, NV.ptr(C), M * N4, N4,
                                  NV.ptr(C), M * N4, NV.ptr(tb), 1, None, None, 0, 0, 0, None, 0, 0, 0, 1, NV.ptr(NV.flag_word()),
                                  NV.stream()) == 0
            torch.cuda.synchronize()
            outs.append(C.cpu().numpy())
    finally:
        L.mvr_set_math(prev)
    assert np.array_equal(outs[0], outs[1])
    ref = A.astype(np.float64) @ B[..., :N].astype(np.float64) + bias[None, :, None] + R[..., :N]
    scale = np.abs(A).astype(np.float64) @ np.abs(B[..., :N]).astype(np.float64) + 1.0
    assert np.all(np.abs(outs[1][..., :N] - ref) <= 1e-5 * scale)


def _big_a_gemm(A, B):
    A[0, 3, 5] = 2.0e3     # x 2^6 past 65504


def _tiny_gemm(A, B):
    A *= 1.0e-7            # every lane's values nonzero but below 2^-9 (B's too: a prologue lifts A)
    B *= 1.0e-7


@pytest.mark.parametrize("edit", [_big_a_gemm, _tiny_gemm])
@pytest.mark.parametrize("combo", [(1, 1, 2, 1, 1), (0, 0, 1, 1, 0), (2, 0, 1, 2, 0)])
def test_gemm_f16_window(gpu, edit, combo):
    """generic GEMM: an operand outside the split-fp16 window re-runs the launch in split-bf16 (bit-identical)"""
    from lib import _native as NV
    pro, bkc, bias, stats, res = combo
    L = NV.lib()
    outs = []
    prev = L.mvr_set_math(0)
    try:
        for f in (0, 1):
            L.mvr_set_math(f)
            outs.append(_run(gpu, 130, 517, 260, 2, pro, bkc, bias, stats, res, seed=3, shared_a=(pro != 1),
                             edit=edit, raw=True))
    finally:
        L.mvr_set_math(prev)
    (c0, s0), (c1, s1) = outs
    assert np.array_equal(c0, c1, equal_nan=True)
    assert s0 is None or np.array_equal(s0, s1, equal_nan=True)


def test_gemm_bf16x3_accuracy_vs_fp32(gpu):
    """The split path's error against float64 stays at plain fp32's level (a float32 BLAS product of the same
    operands)."""
    import torch
    from lib import _native as NV
    r = np.random.RandomState(3)
    M, N, K, b = 128, 2048, 512, 2
    A = r.standard_normal((b, M, K)).astype(np.float32)
    B = r.standard_normal((b, K, N)).astype(np.float32)
    ref = A.astype(np.float64) @ B.astype(np.float64)
    e32 = np.abs((A @ B).astype(np.float64) - ref).max()
    C = torch.empty(b, M, N, device=gpu)
    tA, tB = torch.from_numpy(A).to(gpu), torch.from_numpy(B).to(gpu)
    L = NV.lib()
    assert L.mvr_gemm_f32(M, N, K, b, NV.ptr(tA), M * K, K, NV.ptr(tB), K * N, N, 0, NV.ptr(C), M * N, N, None,
                          0, None, 0, None, None, 0, 0, 0, None, 0, 0, 0, 1, NV.ptr(NV.flag_word()), NV.stream()) == 0
    err = np.abs(C.cpu().numpy() - ref).max()
    assert err < 3 * e32 + 1e-6, (err, e32)


def test_gemm_rejects_bad_layout(gpu):
    import torch
    from lib import _native as NV
    L = NV.lib()
    A = torch.zeros(16, 8, device=gpu)
    B = torch.zeros(8, 16, device=gpu)
    C = torch.zeros(16, 16, device=gpu)
    ok = L.mvr_gemm_f32(16, 16, 8, 1, NV.ptr(A), 0, 8, NV.ptr(B), 0, 16, 0, NV.ptr(C), 0, 16, None, 0, None, 0,
                        None, None, 0, 0, 0, None, 0, 0, 0, 1, NV.ptr(NV.flag_word()), NV.stream())
    assert ok == 0
    # lda not a multiple of 4 / row shorter than round_up(K, 4)
    assert L.mvr_gemm_f32(16, 16, 6, 1, NV.ptr(A), 0, 6, NV.ptr(B), 0, 16, 0, NV.ptr(C), 0, 16, None, 0, None, 0,
                          None, None, 0, 0, 0, None, 0, 0, 0, 1, NV.ptr(NV.flag_word()), NV.stream()) == -1
    # misaligned C
    assert L.mvr_gemm_f32(15, 12, 8, 1, NV.ptr(A), 0, 8, NV.ptr(B), 0, 16, 0, NV.ptr(C[0, 1:]), 0, 16, None, 0,
                          None, 0, None, None, 0, 0, 0, None, 0, 0, 0, 1, NV.ptr(NV.flag_word()), NV.stream()) == -1


@pytest.mark.parametrize("N,K,batch,shared_fold", [(500, 500, 5, False), (500, 500, 300, True), (36, 36, 3, False),
                                                   (300, 260, 4, False), (517, 128, 3, True), (256, 40, 2, False),
                                                   (1, 68, 2, False), (640, 500, 300, False), (200, 512, 7, True)])
def test_oaf_conv2_split_once(gpu, N, K, batch, shared_fold):
    """OAFilter conv2 on the split-once kernel (gemm.hip oaf_conv2_kernel: weight image split once per launch, the
    A slab folded and split once per workgroup, 128 x 256 tiles) against float64 and against the generic kernel:
    ragged N (partial 256-column tiles, an empty second statistics half at N = 517 and 1), K tails, two-stage
    tiles (K = 36, 40: the next tile's fold vectors stored at once) and the largest K (512), more tiles than
    workgroups (batch 300: every workgroup runs several tiles across the stage ring), the eval-mode fold shared
    by every pair (sPb = 0) and per-pair folds (train)."""
    import torch
    from lib import _native as NV
    M = 128
    r = np.random.RandomState(N * 7 + K + batch)
    K4, N4 = r4(K), r4(N)
    A = r.standard_normal((batch, M, K)).astype(np.float32)
    W = (r.standard_normal((N, K)) / np.sqrt(K)).astype(np.float32)
    Rm = r.standard_normal((batch, M, N)).astype(np.float32)
    bias = r.standard_normal(N).astype(np.float32)
    nf = 1 if shared_fold else batch
    sc = r.uniform(0.5, 1.5, (nf, K)).astype(np.float32)
    sh = r.uniform(-0.5, 0.5, (nf, K)).astype(np.float32)
    Ad = np.maximum(A.astype(np.float64) * sc[:, None, :] + sh[:, None, :], 0)
    Cref = Ad @ W.astype(np.float64).T + bias[None, None, :] + Rm
    scale = np.abs(Ad) @ np.abs(W.astype(np.float64)).T + 1.0
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(gpu)   # noqa: E731
    tA, tW, tR, tb, tsc, tsh = t(_pad(A, K4)), t(_pad(W, K4)), t(_pad(Rm, N4)), t(bias), t(sc), t(sh)
    nT = (N + BT - 1) // BT
    L = NV.lib()
    img = torch.empty(int(L.mvr_oaf_conv2_image_bytes(N, K)) // 4 + 4, device=gpu)
    outs = []
    for new in (1, 0):   # the split-once kernel (128 x 256 tiles); the generic GEMM
        C = torch.full((batch, M, N4), float("nan"), device=gpu)
        st = torch.zeros(batch, nT, M, 2, device=gpu)
        if new:
            rc = L.mvr_oaf_conv2_f32(M, N, K, batch, NV.ptr(tA), M * K4, K4, NV.ptr(tW), K4, NV.ptr(C), M * N4, N4,
                                     NV.ptr(tR), M * N4, NV.ptr(tb), NV.ptr(tsc), NV.ptr(tsh), 0 if shared_fold else K,
                                     NV.ptr(st), M, NV.ptr(img), img.numel() * 4, NV.stream())
        else:
            rc = L.mvr_gemm_f32(M, N, K, batch, NV.ptr(tA), M * K4, K4, NV.ptr(tW), 0, K4, 1, NV.ptr(C), M * N4, N4,
                                NV.ptr(tR), M * N4, NV.ptr(tb), 2, NV.ptr(tsc), NV.ptr(tsh), 0 if shared_fold else K,
                                0, 1, NV.ptr(st), M, 0, 1, 1, None, NV.stream())
        assert rc == 0
        torch.cuda.synchronize()
        Cg = C.cpu().numpy().astype(np.float64)
        assert np.all(np.isfinite(Cg)), "padding columns must be written with finite values"
        Cg = Cg[..., :N]
        assert np.all(np.abs(Cg - Cref) <= 1e-5 * scale), np.max(np.abs(Cg - Cref) / scale)
        S = st.cpu().numpy().astype(np.float64)
        for tt in range(nT):
            blk = Cref[:, :, tt * BT:(tt + 1) * BT]
            np.testing.assert_allclose(S[:, tt, :, 0], blk.sum(-1), rtol=1e-4, atol=1e-3)
            dev2 = ((blk - blk.mean(-1, keepdims=True)) ** 2).sum(-1)
            np.testing.assert_allclose(S[:, tt, :, 1], dev2, rtol=1e-4, atol=1e-3)
        outs.append(Cg)
    # the generic kernel differs only in the MFMA k order inside a 32-k stage
    assert np.all(np.abs(outs[0] - outs[1]) <= 2e-6 * scale), np.max(np.abs(outs[0] - outs[1]) / scale)


def test_oaf_conv2_rejects_other_shapes(gpu):
    import torch
    from lib import _native as NV
    L = NV.lib()
    x = torch.zeros(1 << 16, device=gpu)
    p = NV.ptr(x)
    nb = int(L.mvr_oaf_conv2_image_bytes(64, 64))
    assert nb == 3 * 2 * 256 * 32 * 2
    args = lambda M, K, img_bytes: (M, 64, K, 1, p, 0, 68, p, 68, p, 0, 64, p, 0, p, p, p, 0, p, M, p,   # noqa: E731
                                    img_bytes, NV.stream())
    assert L.mvr_oaf_conv2_f32(*args(64, 64, nb)) == -1       # M != 128
    assert L.mvr_oaf_conv2_f32(*args(128, 66, nb)) == -1      # K % 4
    assert L.mvr_oaf_conv2_f32(*args(128, 32, nb)) == -1      # one stage per tile
    assert L.mvr_oaf_conv2_f32(*args(128, 516, 1 << 20)) == -1   # K > 512
    assert L.mvr_oaf_conv2_f32(*args(128, 64, nb - 16)) == -1  # image scratch too small
    torch.cuda.synchronize()
