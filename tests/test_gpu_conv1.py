"""FCGF conv1 (fcgf.py:118-125: 7^3 stencil, 1 -> 32 channels, eval BN) on the GPU: the brick-tiled
split-bf16 MFMA kernel (mvr_spconv_c1 with out_coords NULL: the output set is the input set) against an
fp64 numpy evaluation over the 7^3 kernel map (random features, BN, ReLU) and against the per-row gather
kernel (mvr_spconv_c1 with explicit output coordinates)."""
import numpy as np
import pytest

from synth import synth_scene_fragments

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def frags():
    f, _ = synth_scene_fragments(3, seed=9, n_pts=60000)
    return f


def _bn(N, dev, bn_on, rng):
    vals = (rng.uniform(0.5, 1.5, 32), rng.standard_normal(32), rng.standard_normal(32), rng.uniform(0.5, 2.0, 32))
    vals = [v.astype(np.float32) for v in vals]
    keep = [dev(v) for v in vals]
    p = N.BnP(*[N.ptr(t) for t in keep]) if bn_on else N.BnP(None, None, None, None)
    return p, vals, keep


def _run(gpu, frags, relu, bn_on):
    import torch
    from lib import _native as N
    from lib.sparse import voxelize, CoordinateManager
    c, _, _, _ = voxelize(frags, 0.025, gpu)
    cm = CoordinateManager(c, len(frags))
    M = c.shape[0]
    rng = np.random.default_rng(7)
    feat = rng.standard_normal((M, 1)).astype(np.float32)
    W = (rng.standard_normal((343, 1, 32)) * 0.1).astype(np.float32)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    bnp, (gamma, beta, mean, var), _keep = _bn(N, dev, bn_on, rng)

    nbr = cm.kernel_map("s1", 1, ks=7).cpu().numpy()
    g = np.where(nbr >= 0, feat[np.maximum(nbr, 0), 0].astype(np.float64), 0.0)      # [M, 343]
    ref = g @ W[:, 0, :].astype(np.float64)
    if bn_on:
        ref = (ref - mean) / np.sqrt(var.astype(np.float64) + 1e-5) * gamma + beta
    if relu:
        ref = np.maximum(ref, 0.0)

    fd, Wd = dev(feat), dev(W)
    bricks = cm.brick_map(1)
    L = N.lib()
    out = torch.full((M, 32), float("nan"), device=gpu)
    N.check(L.mvr_spconv_c1(None, M, N.ptr(bricks), M, bricks.numel(), N.ptr(fd), 7, 1, N.ptr(Wd), 32, bnp, 1e-5,
                            int(relu), N.ptr(out), 32, N.stream()), "mvr_spconv_c1 (bricks)")
    old = torch.full((M, 32), float("nan"), device=gpu)
    N.check(L.mvr_spconv_c1(N.ptr(c), M, N.ptr(bricks), M, bricks.numel(), N.ptr(fd), 7, 1, N.ptr(Wd), 32, bnp,
                            1e-5, int(relu), N.ptr(old), 32, N.stream()), "mvr_spconv_c1 (rows)")
    torch.cuda.synchronize()
    return out.cpu().numpy(), old.cpu().numpy(), ref


@pytest.mark.parametrize("relu,bn_on", [(0, True), (1, True), (0, False)])
def test_conv1_bricks_match_fp64(gpu, frags, relu, bn_on):
    out, old, ref = _run(gpu, frags, relu, bn_on)
    assert np.isfinite(out).all(), "rows left unwritten"
    scale = max(1.0, float(np.abs(ref).max()))
    assert np.abs(out - ref).max() <= 2e-5 * scale, np.abs(out - ref).max()
    assert np.abs(old - ref).max() <= 2e-5 * scale, np.abs(old - ref).max()


def test_conv1_bricks_argument_checks(gpu, frags):
    import torch
    from lib import _native as N
    from lib.sparse import voxelize, CoordinateManager
    c, _, _, _ = voxelize(frags[:1], 0.025, gpu)
    cm = CoordinateManager(c, 1)
    M = c.shape[0]
    bricks = cm.brick_map(1)
    f = torch.ones(M, 1, device=gpu)
    W = torch.zeros(343, 1, 32, device=gpu)
    out = torch.empty(M, 32, device=gpu)
    L = N.lib()
    nob = N.BnP(None, None, None, None)

    def call(Mout, ks, step):
        return L.mvr_spconv_c1(None, Mout, N.ptr(bricks), M, bricks.numel(), N.ptr(f), ks, step, N.ptr(W), 32, nob,
                               1e-5, 0, N.ptr(out), 32, N.stream())
    assert call(M - 1, 7, 1) == -1     # the self mode needs Mout == Min
    assert call(M, 5, 1) == -1         # 7^3 only
    assert call(M, 7, 2) == -1         # stride 1 only
    assert call(M, 7, 1) == 0
    torch.cuda.synchronize()
