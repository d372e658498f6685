"""Fused PointCN (csrc/pointcn.hip, lib/filtering/oanet.py:18-43 with an identity shortcut) against
a float64 torch statement on the same inputs: y = W7 relu(t sc2 + sh2) + b7 + x,
t = W3 relu(x sc1 + sh1) + b3, out of place and in place, ragged N, and the per-32-point-chunk
(sum, squared deviations) partials.  Tolerance: fp32-level (split-bf16 MFMA), 2e-5 of the scale."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

C = 128


@pytest.mark.parametrize("P,N,inplace", [(3, 1234, False), (2, 37, True), (1, 5000, True), (5, 5, False)])
def test_pointcn_fused_matches_fp64(gpu, P, N, inplace):
    import torch
    from lib import _native as NV
    r = np.random.RandomState(N + P)
    ld = (N + 3) // 4 * 4
    x = np.zeros((P, C, ld), np.float32)
    x[:, :, :N] = r.standard_normal((P, C, N))
    sc1, sc2 = (r.uniform(0.5, 1.5, (P, C)).astype(np.float32) for _ in range(2))
    sh1, sh2 = (r.uniform(-0.5, 0.5, (P, C)).astype(np.float32) for _ in range(2))
    W3, W7 = ((0.1 * r.standard_normal((C, C))).astype(np.float32) for _ in range(2))
    b3, b7 = ((0.1 * r.standard_normal(C)).astype(np.float32) for _ in range(2))
    d = lambda a: torch.from_numpy(a).double()
    xx = d(x[:, :, :N])
    t = d(W3) @ torch.relu(xx * d(sc1)[:, :, None] + d(sh1)[:, :, None]) + d(b3)[None, :, None]
    ref = (d(W7) @ torch.relu(t * d(sc2)[:, :, None] + d(sh2)[:, :, None]) + d(b7)[None, :, None] + xx).numpy()
    g = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    gx = g(x)
    gy = gx if inplace else torch.full_like(gx, float("nan"))
    nch = (N + 31) // 32
    st = torch.zeros(P, nch, C, 2, device=gpu)
    a = [g(v) for v in (sc1, sh1, sc2, sh2, W3, b3, W7, b7)]
    assert NV.lib().mvr_pointcn_fused(NV.ptr(gx), C * ld, ld, NV.ptr(gy), C * ld, ld, *[NV.ptr(v) for v in a], P, C, N,
                                      NV.ptr(st), C, 0, NV.stream()) == 0
    torch.cuda.synchronize()
    y = gy.cpu().numpy()
    scale = np.abs(ref).max()
    np.testing.assert_allclose(y[:, :, :N], ref, atol=2e-5 * scale, rtol=0)
    assert np.all(y[:, :, N:] == 0)
    s = st.cpu().numpy()
    for k in range(nch):
        blk = ref[:, :, 32 * k:min(N, 32 * k + 32)]
        np.testing.assert_allclose(s[:, k, :, 0], blk.sum(-1), atol=2e-5 * scale * 32, rtol=0)
        np.testing.assert_allclose(s[:, k, :, 1], ((blk - blk.mean(-1, keepdims=True)) ** 2).sum(-1), rtol=1e-4,
                                   atol=1e-6 * scale ** 2 * 32)
