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


@pytest.mark.parametrize("n,m", [(1000, 1500), (33, 4097)])
def test_soft_gumbel_vs_oracle(gpu, n, m, monkeypatch):
    """soft_gumbel (lib/layers.py:72-78, F.gumbel_softmax(-dist, tau, hard=st)): the HIP path's counter-based noise
    restated in oracle/soft_nn.py (float64), soft weights and the straight-through forward value, through Soft_NN and
    the pair-indexed matcher; the noise depends on the fragment pair, not on the batch position.  (The reference's
    own noise comes from torch's RNG and cannot be replayed: parity by restatement)"""
    import torch
    from lib.layers import Soft_NN
    from oracle.soft_nn import soft_nn_gumbel
    B = 3
    L = max(n, m)
    f = unit_features(B, L, 32, seed=7 + n)
    x = np.random.RandomState(9).uniform(-2, 2, (B, L, 3)).astype(np.float32)
    tf, tx = torch.from_numpy(f).to(gpu), torch.from_numpy(x).to(gpu)
    seed = 0x1234_5678_9ABC
    for st in (False, True):
        nn = Soft_NN(corr_type="soft_gumbel", st=st).to(gpu)
        monkeypatch.setattr(nn, "_gumbel_seed", lambda: seed)
        got = nn(tf[:, :n].contiguous(), tf[:, :m].contiguous(), tx[:, :m].contiguous()).cpu().numpy()
        ref = soft_nn_gumbel(f[:, :n], f[:, :m], x[:, :m], np.arange(B), np.arange(B), seed, st=st)
        if not st:
            np.testing.assert_allclose(got, ref, atol=2e-4)
        else:   # the noisy argmax: exact up to fp32 near-ties of the noisy logits
            bad = np.any(np.abs(got - ref) > 1e-6, axis=-1)
            assert bad.mean() < 2e-3, bad.mean()
    # the pair-indexed form (the pipeline's match_pairs): pair (s, t) gets the noise of fragments (s, t)
    pairs = torch.tensor([[0, 1], [2, 0], [1, 1]], dtype=torch.int64, device=gpu)
    out = torch.empty(3, n, 6, device=gpu)
    nn = Soft_NN(corr_type="soft_gumbel", st=False).to(gpu)
    monkeypatch.setattr(nn, "_gumbel_seed", lambda: seed)
    if n == m:
        nn.match_pairs(tf[:, :n].contiguous(), tx[:, :n].contiguous(), pairs, out, n * 6, 6)
        p = pairs.cpu().numpy()
        ref = soft_nn_gumbel(f[p[:, 0], :n], f[p[:, 1], :n], x[p[:, 1], :n], p[:, 0], p[:, 1], seed)
        np.testing.assert_allclose(out[..., 3:].cpu().numpy(), ref, atol=2e-4)


def test_soft_gumbel_hard_picks_follow_softmax(gpu):
    """The Gumbel-max property the mode rests on: the straight-through pick of target j has probability
    softmax(-d)_j (F.gumbel_softmax adds the noise to the logits -d before dividing by tau).  One query against 8 targets, 20000 independent draws (fragment pairs of one batch call)."""
    import torch
    from lib import _native as NV
    P, M = 20000, 8
    fq = unit_features(1, 1, 32, seed=1)[0, 0]
    ft = unit_features(1, M, 32, seed=2)[0]
    F = np.zeros((P + 1, M, 32), np.float32)
    F[0, 0] = fq
    F[1:] = ft                                    # fragment 0: the query; fragments 1..P: the same targets
    X = np.zeros((P + 1, M, 3), np.float32)
    X[:, :, 0] = np.arange(M, dtype=np.float32)   # x coordinate = target index
    pairs = np.stack([np.zeros(P, np.int64), np.arange(1, P + 1)], 1)
    tF, tX, tp = (torch.from_numpy(a).to(gpu) for a in (F, X, pairs))
    out = torch.empty(P, 1, 3, device=gpu)
    tau = 0.5
    rc = NV.lib().mvr_feat_nn_gumbel(NV.ptr(tF), M * 32, NV.ptr(tF), M * 32, None, 0, NV.ptr(tX), M * 3, NV.ptr(tp), P,
                                     1, M, 32, 1.0 / tau, 1, 99, NV.ptr(out), 3, 3, None, NV.stream())
    assert rc == 0
    picks = out[:, 0, 0].cpu().numpy().astype(int)
    d = ((fq[None] - ft) ** 2).sum(-1).astype(np.float64)
    pz = np.exp(-(d - d.min()))   # argmax((-d + g) / tau) = argmax(-d + g): tau does not enter the picks
    pz /= pz.sum()
    freq = np.bincount(picks, minlength=M) / P
    assert np.all(np.abs(freq - pz) < 5 * np.sqrt(pz * (1 - pz) / P) + 1e-3), (freq, pz)
