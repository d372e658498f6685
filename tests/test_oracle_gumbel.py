"""CPU checks of the soft_gumbel restatement (oracle/soft_nn.py gumbel_noise): the counter-based noise is standard
Gumbel (mean = Euler's gamma, variance = pi^2 / 6), uncorrelated across targets, queries and fragment pairs, and
deterministic in its key."""
import numpy as np

from oracle.soft_nn import gumbel_noise, soft_nn_gumbel


def test_gumbel_noise_distribution():
    g = gumbel_noise(12345, 3, 7, 400, 500)
    assert g.shape == (400, 500)
    assert abs(g.mean() - 0.5772156649) < 0.01
    assert abs(g.var() - np.pi ** 2 / 6) < 0.03
    # CDF exp(-exp(-g)) is uniform
    u = np.sort(np.exp(-np.exp(-g.ravel())))
    assert np.abs(u - (np.arange(u.size) + 0.5) / u.size).max() < 0.005
    # neighbouring targets / queries / pairs / seeds are uncorrelated
    for a, b in ((g[:, :-1], g[:, 1:]), (g[:-1], g[1:]), (g, gumbel_noise(12345, 3, 8, 400, 500)),
                 (g, gumbel_noise(12345, 4, 7, 400, 500)), (g, gumbel_noise(12346, 3, 7, 400, 500))):
        assert abs(np.corrcoef(a.ravel(), b.ravel())[0, 1]) < 0.01
    np.testing.assert_array_equal(g, gumbel_noise(12345, 3, 7, 400, 500))


def test_soft_nn_gumbel_limits():
    """without noise the restatement is the soft mode; at a very low temperature the soft weights approach the
    straight-through one-hot"""
    rng = np.random.default_rng(0)
    xf = rng.standard_normal((1, 50, 32)).astype(np.float32)
    yf = rng.standard_normal((1, 60, 32)).astype(np.float32)
    yc = rng.standard_normal((1, 60, 3)).astype(np.float32)
    hard = soft_nn_gumbel(xf, yf, yc, [0], [1], 5, st=True)
    cold = soft_nn_gumbel(xf, yf, yc, [0], [1], 5, st=False, temp=1e-3, min_temp=1e-6)
    np.testing.assert_allclose(cold, hard, atol=1e-6)
