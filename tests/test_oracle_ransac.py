"""RANSAC restatement (oracle/ransac.py = lib/utils.py:671-709 -> Open3D 0.9
registration_ransac_based_on_correspondence; Open3D is absent here, so parity against it is
unpinned): known-answer checks on synthetic correspondences with a known rigid motion, the
Umeyama fit against the reference's own Kabsch restatement (oracle/kabsch.py, lib/utils.py:164-237),
and the draw stream's bounds."""
import numpy as np

from oracle import ransac as O
from oracle.kabsch import kabsch
from synth import random_rotation


def _corr(n, inl, seed, noise=0.005):
    rng = np.random.default_rng(seed)
    R, t = random_rotation(rng), rng.normal(0, 1.0, 3)
    x1 = rng.uniform(-1.5, 1.5, (n, 3))
    x2 = x1 @ R.T + t + np.clip(rng.normal(0, noise, (n, 3)), -0.025, 0.025)
    k = int(round(n * inl))
    out = rng.permutation(n)[k:]
    x2[out] = rng.uniform(-1.5, 1.5, (len(out), 3)) + t
    return x1, x2, R, t, n - len(out)


def test_draws_in_range_and_reproducible():
    d = [O.draws(7, p, it, 4, 13) for p in range(3) for it in range(50)]
    assert all(0 <= i < 13 for row in d for i in row)
    assert d == [O.draws(7, p, it, 4, 13) for p in range(3) for it in range(50)]
    assert O.draws(7, 0, 0, 4, 1000) != O.draws(8, 0, 0, 4, 1000)
    assert O.draws(7, 0, 0, 4, 1000) != O.draws(7, 1, 0, 4, 1000)


def test_umeyama_equals_reference_kabsch():
    rng = np.random.default_rng(0)
    for _ in range(20):
        s = rng.normal(size=(4, 3))
        R0 = random_rotation(rng)
        d = s @ R0.T + rng.normal(size=3) + rng.normal(0, 0.01, (4, 3))
        R, t = O.umeyama(s, d)
        Rk, tk, _, _ = kabsch(s[None], d[None])
        np.testing.assert_allclose(R, Rk[0], atol=1e-12)
        np.testing.assert_allclose(t, tk[0, :, 0], atol=1e-12)
        assert abs(np.linalg.det(R) - 1) < 1e-12


def test_recovers_known_motion():
    x1, x2, R, t, k = _corr(400, 0.3, seed=1)
    T, fit, rmse, b, _, cnt, _ = O.ransac(x1, x2, seed=3, iters=300)
    assert b >= 0 and cnt[b] == int(round(fit * 400))
    assert abs(fit - k / 400) < 0.02
    np.testing.assert_allclose(T[:3, :3], R, atol=2e-2)
    np.testing.assert_allclose(T[:3, 3], t, atol=3e-2)
    assert 0 < rmse < 0.05


def test_degenerate_inputs_give_identity():
    x = np.zeros((3, 3))
    T, fit, rmse, b, *_ = O.ransac(x, x, iters=10)
    assert b == -1 and fit == 0.0 and rmse == 0.0 and np.array_equal(T, np.eye(4))
