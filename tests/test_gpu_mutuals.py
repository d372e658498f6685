"""knn_point(k=1) / extract_mutuals on the device (csrc/knn.hip) against the reference's own outputs
(tests/golden/mutuals.npz: /root/reference/lib/utils.py:274-299, :822-848) and, at the full pair size
(5000 x 5000 per pair), against oracle/mutuals.py on the same seeded inputs.  Integer / flag outputs are bit-exact;
the fp32 distances are the reference's own expression evaluated in its order, so they match exactly too."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _t(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def test_knn_point_golden(gpu):
    from lib.utils import knn_point
    g = golden("mutuals.npz")
    d, i = knn_point(1, _t(g["x2"], gpu), _t(g["x1m"], gpu))
    np.testing.assert_array_equal(i.cpu().numpy(), g["knn1_i"])
    np.testing.assert_array_equal(d.cpu().numpy(), g["knn1_d"])
    d3, i3 = knn_point(3, _t(g["x2"], gpu), _t(g["x1m"][:, :50], gpu))
    np.testing.assert_array_equal(i3.cpu().numpy(), g["knn3_i"])
    np.testing.assert_array_equal(d3.cpu().numpy(), g["knn3_d"])


def test_extract_mutuals_golden(gpu):
    from lib.utils import extract_mutuals
    g = golden("mutuals.npz")
    m = extract_mutuals(*[_t(g[k], gpu) for k in ("x1", "x2", "x1m", "x2m")])
    np.testing.assert_array_equal(m.cpu().numpy(), g["mutuals"])


@pytest.mark.parametrize("n", [1, 1023, 1025, 5000])
def test_extract_mutuals_vs_oracle_strided(gpu, n):
    """The fused xs buffer layout (x_s | x_corr, row stride 6) as lib.pairwise passes it, ragged tile edges."""
    import torch
    from lib.utils import extract_mutuals
    from oracle.mutuals import mutuals
    r = np.random.RandomState(n)
    B = 3
    xs = r.uniform(-1, 1, (B, n, 6)).astype(np.float32)
    x2 = r.uniform(-1, 1, (B, n, 3)).astype(np.float32)
    back = (xs[..., :3] + r.normal(0, 0.03, (B, n, 3))).astype(np.float32)
    perm = np.stack([r.permutation(n) for _ in range(B)])
    x2m = np.empty_like(back)
    for b in range(B):
        x2m[b, perm[b]] = back[b]
        xs[b, :, 3:] = x2[b, perm[b]] + r.normal(0, 1e-3, (n, 3))
    X = torch.from_numpy(xs).to(gpu)
    m = extract_mutuals(X[..., :3], _t(x2, gpu), X[..., 3:], _t(x2m, gpu))
    ref, _ = mutuals(xs[..., :3], x2, xs[..., 3:], x2m)
    np.testing.assert_array_equal(m.cpu().numpy(), ref)


def test_knn1_ties_first_index(gpu):
    from lib.utils import knn_point
    pts = np.zeros((1, 10, 3), np.float32)
    pts[0, :, 0] = [3, 1, 2, 1, 5, 1, 7, 8, 9, 1]     # four targets at distance 0 from the query
    q = np.asarray([[[1, 0, 0]]], np.float32)
    d, i = knn_point(1, _t(pts, gpu), _t(q, gpu))
    assert int(i.item()) == 1 and float(d.item()) == 0.0
