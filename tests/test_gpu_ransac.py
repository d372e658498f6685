"""Batched GPU RANSAC (csrc/procrustes.hip mvr_ransac, lib/utils.py run_ransac[_batch]) against the
restatement of lib/utils.py:671-709 / Open3D 0.9 in oracle/ransac.py (Open3D itself: parity unpinned):
  * every hypothesis (same counter-stream draws, Umeyama fit) within 1e-9 of the oracle's numpy-SVD fit;
  * inlier counts / error sums of the GPU's own hypotheses, re-evaluated by the oracle in the kernel's fp64
    operation order: the selected iteration, fitness and rmse identical (bit for bit);
  * ragged per-pair counts (n < ransac_n -> identity, fitness 0), batch == per-pair calls;
  * full size (5000 correspondences, 2500 iterations): the known motion is recovered."""
import numpy as np
import pytest

from oracle import ransac as O
from synth import random_rotation

pytestmark = pytest.mark.gpu


def _corr(n, inl, seed, noise=0.005):
    rng = np.random.default_rng(seed)
    R, t = random_rotation(rng), rng.normal(0, 1.0, 3)
    x1 = rng.uniform(-1.5, 1.5, (n, 3))
    x2 = x1 @ R.T + t + np.clip(rng.normal(0, noise, (n, 3)), -0.025, 0.025)
    out = rng.permutation(n)[int(round(n * inl)):]
    x2[out] = rng.uniform(-1.5, 1.5, (len(out), 3)) + t
    return x1, x2, R, t


def _gpu(x1, x2, counts, seed, iters, gpu):
    import torch
    from lib import _native as N
    P, n = x1.shape[0], x1.shape[1]
    X1 = torch.from_numpy(x1).to(gpu)
    X2 = torch.from_numpy(x2).to(gpu)
    cnt = torch.tensor(counts, dtype=torch.int32, device=gpu)
    T = torch.empty(P, 4, 4, dtype=torch.float64, device=gpu)
    fit, rmse = (torch.empty(P, dtype=torch.float64, device=gpu) for _ in range(2))
    best = torch.empty(P, dtype=torch.int32, device=gpu)
    hyp = torch.empty(P, iters, 12, dtype=torch.float64, device=gpu)
    L = N.lib()
    ws = torch.empty(L.mvr_ransac_workspace_bytes(P, iters), dtype=torch.uint8, device=gpu)
    assert L.mvr_ransac(N.ptr(X1), N.ptr(X2), n * 3, N.ptr(cnt), P, 4, iters, 0.05, seed, N.ptr(T), N.ptr(fit),
                        N.ptr(rmse), N.ptr(best), N.ptr(hyp), N.ptr(ws), ws.numel(), N.stream()) == 0
    torch.cuda.synchronize()
    return T.cpu().numpy(), fit.cpu().numpy(), rmse.cpu().numpy(), best.cpu().numpy(), hyp.cpu().numpy()


@pytest.mark.parametrize("n,iters", [(300, 256), (1000, 700), (37, 100)])
def test_ransac_matches_oracle(gpu, n, iters):
    P = 3
    data = [_corr(n, f, seed=10 + p) for p, f in enumerate((0.05, 0.3, 0.8))]
    x1 = np.stack([d[0] for d in data])
    x2 = np.stack([d[1] for d in data])
    counts = [n, n - 5, n // 2]
    T, fit, rmse, best, hyp = _gpu(x1, x2, counts, 11, iters, gpu)
    for p in range(P):
        m = counts[p]
        To, fo, ro, bo, own, _, _ = O.ransac(x1[p, :m], x2[p, :m], seed=11, iters=iters, p=p, hyps=hyp[p])
        # the fits themselves: GPU Jacobi SVD vs numpy LAPACK on the same draws (draws with fewer than three
        # distinct correspondences have a rank-1 covariance: the rotation is not unique, skip them)
        ok = [it for it in range(iters) if len(set(O.draws(11, p, it, 4, m))) >= 3]
        assert len(ok) > 0.9 * iters
        np.testing.assert_allclose(hyp[p][ok], own[ok], atol=1e-9)
        # the selection over the GPU's hypotheses, re-evaluated on the host: identical
        assert best[p] == bo, (p, best[p], bo)
        assert fit[p] == fo and rmse[p] == ro, (p, fit[p], fo, rmse[p], ro)
        assert np.array_equal(T[p], To)


def test_ragged_and_degenerate(gpu):
    x1, x2, _, _ = _corr(64, 0.5, seed=3)
    x1 = np.stack([x1] * 4)
    x2 = np.stack([x2] * 4)
    T, fit, rmse, best, _ = _gpu(x1, x2, [0, 3, 4, 64], 5, 64, gpu)
    for p in (0, 1):   # fewer correspondences than ransac_n: Open3D returns RegistrationResult()
        assert best[p] == -1 and fit[p] == 0.0 and rmse[p] == 0.0 and np.array_equal(T[p], np.eye(4))
    assert best[2] >= 0 and fit[2] > 0 and best[3] >= 0


def test_batch_equals_single_calls(gpu):
    """run_ransac_batch: pair p draws from counter stream p; each pair equals the oracle's single-pair run"""
    from lib.utils import run_ransac_batch
    data = [_corr(500, 0.25, seed=s) for s in range(4)]
    x1 = np.stack([d[0] for d in data])
    x2 = np.stack([d[1] for d in data])
    Tb = run_ransac_batch(x1, x2, seed=9, iters=300)
    for p in range(4):
        To = O.ransac(x1[p], x2[p], seed=9, iters=300, p=p)[0]
        np.testing.assert_allclose(Tb[p], To, atol=1e-9)
        T1 = _gpu(x1[p:p + 1], x2[p:p + 1], [500], 9, 300, gpu)[0][0]   # alone: counter stream 0
        np.testing.assert_allclose(T1, O.ransac(x1[p], x2[p], seed=9, iters=300, p=0)[0], atol=1e-9)


def test_run_ransac_full_size_recovers_motion(gpu):
    from lib.utils import run_ransac
    x1, x2, R, t = _corr(5000, 0.15, seed=21)
    T = run_ransac(x1.astype(np.float32), x2.astype(np.float32), seed=1)   # reference call shape: [n,3] each
    assert T.shape == (4, 4) and T.dtype == np.float64
    np.testing.assert_allclose(T[:3, :3], R, atol=1e-2)
    np.testing.assert_allclose(T[:3, 3], t, atol=2e-2)
    np.testing.assert_allclose(T[3], [0, 0, 0, 1])
