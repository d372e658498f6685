"""Fused feature-NN kernel (mvr_feat_nn) and the Sampler gather vs the
reference's golden vectors (lib/layers.py Soft_NN / Sampler) and the oracle."""
import numpy as np
import pytest

from conftest import golden
from synth import unit_features

pytestmark = pytest.mark.gpu


def test_soft_nn_golden_modes(gpu):
    import torch
    from lib.layers import Soft_NN
    g = golden("softnn.npz")
    fs, ft, yc = (torch.from_numpy(g[k]).to(gpu) for k in ("fs", "ft", "yc"))
    for (mode, st), key, tol in ((("soft", False), "x_soft", 2e-5), (("soft", True), "x_soft_st", 0),
                                 (("hard", False), "x_hard", 0)):
        nn = Soft_NN(corr_type=mode, st=st).to(gpu)
        x = nn(fs, ft, yc).cpu().numpy()
        np.testing.assert_allclose(x, g[key], atol=tol + 1e-7)
    nn = Soft_NN(corr_type="soft", st=False, temp=0.005).to(gpu)      # tau^2 clamped at min_temp
    np.testing.assert_allclose(nn(fs, ft, yc).cpu().numpy(), g["x_soft_cold"], atol=2e-3)


@pytest.mark.parametrize("n,m", [(5000, 5000), (1000, 777), (33, 4097)])
def test_feat_nn_pairs_vs_oracle(gpu, n, m):
    """fragment/pair-indexed form used by the pipeline (no [P,n,m] tensor)."""
    import torch
    from lib import _native as NV
    from oracle.soft_nn import soft_nn
    B = 4
    L = max(n, m)
    f = unit_features(B, L, 32, seed=n + m)
    x = np.random.RandomState(5).uniform(-2, 2, (B, L, 3)).astype(np.float32)
    pairs = np.array([[0, 1], [2, 3], [3, 0], [1, 1]], dtype=np.int64)
    tf, tx, tp = (torch.from_numpy(a).to(gpu) for a in (f, x, pairs))
    out = torch.empty(len(pairs), n, 6, device=gpu)
    for mode in (0, 1):
        rc = NV.lib().mvr_feat_nn(NV.ptr(tf), L * 32, NV.ptr(tf), L * 32, NV.ptr(tx), L * 3, NV.ptr(tx), L * 3,
                                  NV.ptr(tp), len(pairs), n, m, 32, 1.0 / 0.09, mode, NV.ptr(out), n * 6, 6, None,
                                  NV.stream())
        assert rc == 0
        o = out.cpu().numpy()
        ref = soft_nn(f[pairs[:, 0], :n], f[pairs[:, 1], :m], x[pairs[:, 1], :m], "soft", st=(mode == 1))
        np.testing.assert_array_equal(o[..., :3], x[pairs[:, 0], :n])
        if mode == 0:
            np.testing.assert_allclose(o[..., 3:], ref, atol=3e-5)
        else:  # exact argmax except fp32 near-ties (distance gap < rounding)
            bad = np.any(o[..., 3:] != ref, axis=-1)
            assert bad.mean() < 1e-3, bad.mean()


@pytest.mark.parametrize("scale,offset", [(1.0, 0.0), (2.5, 0.0), (0.05, 130.0)])
def test_feat_nn_fast_path_matches_online(gpu, scale, offset):
    """Soft mode: the bounded-shift path (feat_nn_fast, split-fp16 and split-bf16 distance MFMAs) against the
    online-softmax path; at scale 2.5 some queries' softmax sums underflow the fast path and their workgroups
    fall back; with a common offset of 150 the descriptors are close together (no underflow) but their norms
    are past the split-fp16 range (|f|^2 >= 2^14): the fp16 form falls back."""
    import torch
    from lib import _native as NV
    from oracle.soft_nn import soft_nn
    B, n = 3, 2000
    f = unit_features(B, n, 32, seed=7)
    f[1] *= np.float32(scale if offset == 0 else 1.0)   # fragment 1 farther from everything in feature space
    if offset:
        f = (f * np.float32(scale) + np.float32(offset / np.sqrt(32))).astype(np.float32)
    x = np.random.RandomState(6).uniform(-2, 2, (B, n, 3)).astype(np.float32)
    pairs = np.array([[0, 1], [1, 2], [2, 0]], dtype=np.int64)
    tf, tx, tp = (torch.from_numpy(a).to(gpu) for a in (f, x, pairs))
    L = NV.lib()
    outs = []
    prev = L.mvr_set_math(0)
    try:
        for math, online in ((1, 0), (0, 0), (0, 1)):   # fast path split-fp16, split-bf16; the online path
            L.mvr_set_math(math)
            with NV.force("feat_nn_online", online):
                out = torch.empty(len(pairs), n, 6, device=gpu)
                rc = L.mvr_feat_nn(NV.ptr(tf), n * 32, NV.ptr(tf), n * 32, NV.ptr(tx), n * 3, NV.ptr(tx), n * 3,
                                   NV.ptr(tp), len(pairs), n, n, 32, 1.0 / 0.09, 0, NV.ptr(out), n * 6, 6, None,
                                   NV.stream())
            assert rc == 0
            outs.append(out.cpu().numpy())
    finally:
        L.mvr_set_math(prev)
    for o in outs:
        assert np.all(np.isfinite(o))
    if offset:   # (|f|^2 ~ 2^14: fp32 distances themselves are off by ~1e-3 here, no oracle comparison)
        assert np.array_equal(outs[0], outs[2])   # every fp16 workgroup fell back to the online path
        return
    ref = soft_nn(f[pairs[:, 0]].astype(np.float64), f[pairs[:, 1]].astype(np.float64),
                  x[pairs[:, 1]].astype(np.float64), "soft", st=False)
    for o in outs:
        np.testing.assert_allclose(o[..., 3:], ref, atol=3e-5)
    np.testing.assert_allclose(outs[0], outs[2], atol=3e-5)
    np.testing.assert_allclose(outs[1], outs[2], atol=3e-5)


def test_sampler_indices_and_gather(gpu):
    import torch
    from lib.layers import Sampler
    g = golden("sampler.npz")
    for tag in ("demo", "short"):
        pts = [int(v) for v in g["pts_" + tag]]
        tot = sum(pts)
        C = torch.zeros(tot, 3, device=gpu)
        C[:, 0] = torch.arange(tot, device=gpu, dtype=torch.float32)
        F = torch.randn(tot, 32, device=gpu)
        np.random.seed(41)
        sc, sf = Sampler("rand", 5000)(C, F, torch.tensor(pts))
        idx = sc[..., 0].long()
        assert np.array_equal(idx.cpu().numpy(), g["idx_" + tag])
        assert torch.equal(sf, F[idx])


@pytest.mark.parametrize("n,m,scale", [(5000, 5000, 1.0), (1000, 777, 1.0), (33, 4097, 1.0), (2000, 2000, 2.5)])
def test_feat_nn_presplit_image_identical(gpu, n, m, scale):
    """mvr_feat_nn_ws (targets split once per call into an image of the LDS stages, staged by LDS-DMA) against
    mvr_feat_nn (each workgroup loads and splits its stages): bit-identical outputs, soft and argmax modes, ragged
    target counts (partial last stage), fragments whose softmax sums underflow (workgroup fallback, scale 2.5)"""
    import torch
    from lib import _native as NV
    B = 4
    L_ = max(n, m)
    f = unit_features(B, L_, 32, seed=n + m + 1)
    f[1] *= np.float32(scale)
    x = np.random.RandomState(9).uniform(-2, 2, (B, L_, 3)).astype(np.float32)
    pairs = np.array([[0, 1], [2, 3], [3, 0], [1, 1], [1, 2]], dtype=np.int64)
    tf, tx, tp = (torch.from_numpy(a).to(gpu) for a in (f, x, pairs))
    L = NV.lib()
    nb = L.mvr_feat_nn_workspace_bytes(B, m)
    ws = torch.empty(nb, dtype=torch.uint8, device=gpu)
    for mode in (0, 1):
        outs = []
        for use_ws in (False, True):
            out = torch.full((len(pairs), n, 6), float("nan"), device=gpu)
            args = (NV.ptr(tf), L_ * 32, NV.ptr(tf), L_ * 32, NV.ptr(tx), L_ * 3, NV.ptr(tx), L_ * 3, NV.ptr(tp),
                    len(pairs), n, m, 32, 1.0 / 0.09, mode, NV.ptr(out), n * 6, 6, None)
            rc = (L.mvr_feat_nn_ws(*args, B, NV.ptr(ws), nb, NV.stream()) if use_ws
                  else L.mvr_feat_nn(*args, NV.stream()))
            assert rc == 0
            outs.append(out.cpu().numpy())
        assert np.array_equal(outs[0], outs[1]), np.nanmax(np.abs(outs[0] - outs[1]))
    assert L.mvr_feat_nn_ws(*args, B, NV.ptr(ws), nb - 16, NV.stream()) == -1   # workspace too small
