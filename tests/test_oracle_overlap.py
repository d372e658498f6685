"""Overlap-gate oracle (oracle/overlap.py, lib/utils.py:713-786) against known answers: Open3D's
VoxelDownSample anchoring / centroid rule on hand-made points, and the NN ratio on exact and
shifted copies."""
import numpy as np

from oracle.overlap import voxel_down_sample, compute_overlap_ratio, overlap_counts


def test_voxel_down_sample_known_answer():
    v = 1.0
    # min bound (0,0,0) -> grid anchored at -0.5: cells [-0.5,0.5), [0.5,1.5), ...
    p = np.array([[0.0, 0.0, 0.0], [0.4, 0.0, 0.0], [0.6, 0.0, 0.0], [1.4, 0.2, 0.0], [0.1, 0.1, 0.1]])
    c = voxel_down_sample(p, v)
    c = c[np.lexsort(c.T[::-1])]
    np.testing.assert_allclose(c, [[(0.0 + 0.4 + 0.1) / 3, 0.1 / 3, 0.1 / 3], [1.0, 0.1, 0.0]])


def test_overlap_identity_and_shift():
    r = np.random.default_rng(0)
    pc = r.uniform(0, 2, (2000, 3))
    assert compute_overlap_ratio(pc, pc, np.eye(4), method="3DMatch") == 1.0
    T = np.eye(4)
    T[0, 3] = 10.0                    # far apart: nothing matches
    assert compute_overlap_ratio(pc, pc, T, method="3DMatch") == 0.0
    m01, m10, ni, nj = overlap_counts(pc, pc[:500], np.eye(4), method="3DMatch")
    assert m10 == 500 and nj == 500 and ni == 2000 and 0 < m01 < 2000
