"""Sampler 'rand' (reference lib/layers.py:145-148): the library's host replay of numpy's legacy
RandomState shuffle (mvr_sample_rand_mt19937) must draw exactly np.random.choice's indices and leave
the global RNG in the same state.  Host-only: runs without a GPU."""
import os

import numpy as np
import pytest

from conftest import PKG

LIB = os.path.join(PKG, "libmvreg_hip.so")


def _reference_draws(pts, tgt):
    out, start = [], 0
    for n in pts:
        out.append(np.random.choice(np.arange(start, start + n), tgt, replace=False))
        start += n
    return np.stack(out)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libmvreg_hip.so not built")
@pytest.mark.parametrize("seed,pts,tgt", [(41, (18977, 19082), 5000), (0, (20393,) * 4, 5000),
                                          (7, (5000, 5001, 7000, 65536, 65537), 5000), (3, (1, 2, 3, 9), 1),
                                          (11, (300, 17, 1000), 17), (5, (4096, 4097), 0)])
def test_rand_sampler_replays_numpy(seed, pts, tgt):
    import torch  # noqa: F401
    from lib.layers import Sampler
    s = Sampler("rand", targeted_num_points=tgt)
    np.random.seed(seed)
    np.random.random(3)                       # a state part-way through a key block
    ours = s.indices(list(pts)).numpy()
    after_ours = np.random.random(4)
    np.random.seed(seed)
    np.random.random(3)
    ref = _reference_draws(pts, tgt)
    after_ref = np.random.random(4)
    assert ours.shape == ref.shape
    assert np.array_equal(ours, ref)
    assert np.array_equal(after_ours, after_ref)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libmvreg_hip.so not built")
def test_rand_sampler_with_replacement_falls_back_to_numpy():
    import torch  # noqa: F401
    from lib.layers import Sampler
    s = Sampler("rand", targeted_num_points=50)
    np.random.seed(2)
    ours = s.indices([40, 60]).numpy()
    np.random.seed(2)
    ref = np.stack([np.random.choice(np.arange(0, 40), 50, replace=True),
                    np.random.choice(np.arange(40, 100), 50, replace=True)])
    assert np.array_equal(ours, ref)
