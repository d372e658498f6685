"""Fused fp32-MFMA GEMM (csrc/gemm.hip) vs a float64 numpy reference, every
prologue/epilogue combination the OANet schedule uses, ragged shapes."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BT = 128  # GEMM tile (csrc/gemm.hpp)


def _run(gpu, M, N, K, batch, pro, bkc, bias_mode, stats_mode, res, seed=0, use_v1=0):
    import torch
    from lib import _native as NV
    r = np.random.RandomState(seed)
    A = r.standard_normal((batch, M, K)).astype(np.float32)
    Bm = r.standard_normal((batch, K, N)).astype(np.float32)       # logical B(k, n)
    Bstore = np.ascontiguousarray(np.swapaxes(Bm, 1, 2)) if bkc else Bm
    R = r.standard_normal((batch, M, N)).astype(np.float32) if res else None
    bias = r.standard_normal(M if bias_mode == 1 else N).astype(np.float32) if bias_mode else None
    sc = sh = None
    if pro in (1, 2):
        sc = r.uniform(0.5, 1.5, (batch, K)).astype(np.float32)
        sh = r.uniform(-0.5, 0.5, (batch, K)).astype(np.float32)
    elif pro == 3:
        sc = r.uniform(0.0, 1.0, (batch, N)).astype(np.float32)     # "max"
        sh = r.uniform(0.5, 1.5, (batch, N)).astype(np.float32)     # "1/sum"
    # reference in float64
    Ad, Bd = A.astype(np.float64), Bm.astype(np.float64)
    if pro == 1:
        Ad = np.maximum(Ad * sc[:, None, :] + sh[:, None, :], 0)
    elif pro == 2:
        Bd = np.maximum(Bd * sc[:, :, None] + sh[:, :, None], 0)
    elif pro == 3:
        Bd = np.exp(Bd - sc[:, None, :]) * sh[:, None, :]
    Cref = Ad @ Bd
    if bias_mode == 1:
        Cref += bias[None, :, None]
    elif bias_mode == 2:
        Cref += bias[None, None, :]
    if res:
        Cref += R
    dev = gpu
    t = lambda x: None if x is None else torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    tA, tB, tR, tb, tsc, tsh = t(A), t(Bstore), t(R), t(bias), t(sc), t(sh)
    C = torch.full((batch, M, N), float("nan"), device=dev)
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
    L = NV.lib()
    rc = L.mvr_gemm_f32_variant(M, N, K, batch, NV.ptr(tA), M * K, K, NV.ptr(tB), K * N, (K if bkc else N), bkc,
                                NV.ptr(C), M * N, N, NV.ptr(tR), M * N, NV.ptr(tb), bias_mode, NV.ptr(tsc),
                                NV.ptr(tsh), (K if pro in (1, 2) else N), pro, NV.ptr(st), st_ld, 0, stats_mode,
                                use_v1, NV.stream())
    assert rc == 0
    torch.cuda.synchronize()
    Cg = C.cpu().numpy().astype(np.float64)
    scale = np.abs(Ad) @ np.abs(Bd) + 1.0
    assert np.all(np.abs(Cg - Cref) <= 1e-5 * scale), np.max(np.abs(Cg - Cref) / scale)
    if st is None:
        return
    S = st.cpu().numpy().astype(np.float64)
    if stats_mode in (1, 2):
        for tt in range(nT):
            blk = Cref[:, :, tt * BT:(tt + 1) * BT]
            if stats_mode == 1:
                np.testing.assert_allclose(S[:, tt, :, 0], blk.sum(-1), rtol=1e-4, atol=1e-3)
                np.testing.assert_allclose(S[:, tt, :, 1], (blk ** 2).sum(-1), rtol=1e-4, atol=1e-3)
            else:
                mx = blk.max(-1)
                np.testing.assert_allclose(S[:, tt, :, 0], mx, rtol=1e-5, atol=1e-5)
                np.testing.assert_allclose(S[:, tt, :, 1], np.exp(blk - mx[..., None]).sum(-1), rtol=1e-4)
    else:
        for tt in range(mT):
            blk = Cref[:, tt * BT:(tt + 1) * BT, :]
            if stats_mode == 4:
                np.testing.assert_allclose(S[:, tt, :, 0], blk.sum(1), rtol=1e-4, atol=1e-3)
                np.testing.assert_allclose(S[:, tt, :, 1], (blk ** 2).sum(1), rtol=1e-4, atol=1e-3)
            else:
                mx = blk.max(1)
                np.testing.assert_allclose(S[:, tt, :, 0], mx, rtol=1e-5, atol=1e-5)
                np.testing.assert_allclose(S[:, tt, :, 1], np.exp(blk - mx[:, None, :]).sum(1), rtol=1e-4)


# (pro, bkc, bias, stats, res) — the dispatch table of csrc/gemm.hip
COMBOS = [(0, 0, 1, 1, 0), (0, 0, 1, 0, 0), (2, 0, 1, 1, 0), (2, 0, 1, 0, 0), (2, 0, 1, 4, 0), (2, 0, 1, 1, 1),
          (2, 0, 1, 2, 0), (2, 0, 1, 3, 0), (3, 1, 0, 1, 0), (3, 0, 0, 1, 0), (1, 1, 2, 1, 1), (0, 0, 0, 0, 0),
          (0, 1, 0, 0, 0)]


@pytest.mark.parametrize("combo", COMBOS)
@pytest.mark.parametrize("shape", [(128, 256, 128, 2), (130, 517, 37, 3), (500, 300, 64, 1), (1, 40, 6, 2),
                                   (130, 516, 36, 3), (256, 1000, 500, 2), (128, 5000, 4, 1)])
@pytest.mark.parametrize("use_v1", [0, 1])
def test_gemm_modes(gpu, combo, shape, use_v1):
    M, N, K, b = shape
    pro, bkc, bias, stats, res = combo
    _run(gpu, M, N, K, b, pro, bkc, bias, stats, res, seed=hash((combo, shape)) % 1000, use_v1=use_v1)


def test_gemm_unaligned_ld_scalar_path(gpu):
    # K=6 rows (conv1 of reg_init) -> A rows not 16-byte aligned
    _run(gpu, 128, 5000, 6, 2, 0, 0, 1, 1, 0)
    _run(gpu, 128, 999, 8, 2, 0, 0, 1, 1, 0)
