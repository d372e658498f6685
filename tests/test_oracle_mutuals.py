"""The mutual-NN oracle (oracle/mutuals.py) against the reference's own outputs (tests/golden/mutuals.npz, made by
tests/golden/make_golden.py from /root/reference/lib/utils.py:274-299 and :822-848)."""
import numpy as np

from conftest import golden
from oracle.mutuals import knn1, mutuals


def test_knn1_matches_reference():
    g = golden("mutuals.npz")
    d, i = knn1(g["x2"], g["x1m"])
    np.testing.assert_array_equal(i, g["knn1_i"][..., 0])
    np.testing.assert_array_equal(d, g["knn1_d"][..., 0])


def test_mutuals_match_reference():
    g = golden("mutuals.npz")
    m, _ = mutuals(g["x1"], g["x2"], g["x1m"], g["x2m"])
    np.testing.assert_array_equal(m, g["mutuals"])
    assert 0.2 < m.mean() < 0.8          # the fixture straddles the threshold
