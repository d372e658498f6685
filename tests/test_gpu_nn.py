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


@pytest.mark.parametrize("scale", [1.0, 2.5])
def test_feat_nn_fast_path_matches_online(gpu, scale):
    """Soft mode: the bounded-shift path (feat_nn_fast) against the online-softmax path; at scale 2.5
    some queries' softmax sums underflow the fast path and their workgroups fall back."""
    import torch
    from lib import _native as NV
    from oracle.soft_nn import soft_nn
    B, n = 3, 2000
    f = unit_features(B, n, 32, seed=7)
    f[1] *= np.float32(scale)           # fragment 1 farther from everything in feature space
    x = np.random.RandomState(6).uniform(-2, 2, (B, n, 3)).astype(np.float32)
    pairs = np.array([[0, 1], [1, 2], [2, 0]], dtype=np.int64)
    tf, tx, tp = (torch.from_numpy(a).to(gpu) for a in (f, x, pairs))
    L = NV.lib()
    outs = []
    for fast in (1, 0):
        prev = L.mvr_set_feat_nn_fast(fast)
        out = torch.empty(len(pairs), n, 6, device=gpu)
        rc = L.mvr_feat_nn(NV.ptr(tf), n * 32, NV.ptr(tf), n * 32, NV.ptr(tx), n * 3, NV.ptr(tx), n * 3, NV.ptr(tp),
                           len(pairs), n, n, 32, 1.0 / 0.09, 0, NV.ptr(out), n * 6, 6, None, NV.stream())
        L.mvr_set_feat_nn_fast(prev)
        assert rc == 0
        outs.append(out.cpu().numpy())
    ref = soft_nn(f[pairs[:, 0]], f[pairs[:, 1]], x[pairs[:, 1]], "soft", st=False)
    assert np.all(np.isfinite(outs[0]))
    np.testing.assert_allclose(outs[0][..., 3:], ref, atol=3e-5)
    np.testing.assert_allclose(outs[0], outs[1], atol=3e-5)


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
