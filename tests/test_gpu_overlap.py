"""GPU overlap gate (csrc/overlap.hip, lib/overlap.py) against the oracle (oracle/overlap.py =
lib/utils.py:713-786 with sklearn's NN as in the reference): Open3D-style voxel centroids
bit-exact, matched-point counts exact, for the 'FCGF' (default in the benchmark) and '3DMatch'
methods, batched over the pairs of a synthetic scene with ground-truth and perturbed transforms."""
import numpy as np
import pytest

from synth import synth_scene_fragments, random_rotation

pytestmark = pytest.mark.gpu


def _scene():
    frags, poses = synth_scene_fragments(n_frag=5, seed=7, n_pts=30000, density=26000.0)
    return frags, poses


def _pairs_trans(poses, seed=3):
    rng = np.random.default_rng(seed)
    pairs, trans = [], []
    for i in range(len(poses)):
        for j in range(i + 1, len(poses)):
            T = np.linalg.inv(poses[i]) @ poses[j]          # fragment j -> fragment i
            if (i + j) % 2:                                   # perturbed estimate
                D = np.eye(4)
                D[:3, :3] = random_rotation(rng) if (i + j) % 3 == 0 else np.eye(3)
                D[:3, 3] = rng.normal(0, 0.05, 3)
                T = T @ D
            pairs.append((i, j))
            trans.append(T)
    return np.array(pairs), np.array(trans)


def test_voxel_centroids_bit_exact(gpu):
    from lib.overlap import FragmentOverlap
    from oracle.overlap import voxel_down_sample
    frags, _ = _scene()
    fo = FragmentOverlap(frags, "FCGF", 0.025)
    c = fo.xyz.cpu().numpy()
    for b, f in enumerate(frags):
        g = c[fo.off[b]:fo.off[b + 1]]
        o = voxel_down_sample(f, 0.025)
        assert g.shape == o.shape
        g = g[np.lexsort(g.T[::-1])]
        o = o[np.lexsort(o.T[::-1])]
        np.testing.assert_array_equal(g, o)


@pytest.mark.parametrize("method", ["FCGF", "3DMatch"])
def test_overlap_counts_match_oracle(gpu, method):
    from lib.overlap import FragmentOverlap, overlap_ratio
    from oracle.overlap import overlap_counts, compute_overlap_ratio
    frags, poses = _scene()
    pairs, trans = _pairs_trans(poses)
    fo = FragmentOverlap(frags, method, 0.025)
    got = fo.counts(pairs, trans)
    ratios = fo.ratios(pairs, trans)
    for k, (i, j) in enumerate(pairs):
        m01, m10, ni, nj = overlap_counts(frags[i], frags[j], trans[k], method, 0.025)
        assert (got[k, 0], got[k, 1]) == (m01, m10), (k, i, j)
        assert ratios[k] == max(m01 / ni, m10 / nj)
    assert ratios.max() > 0.3 and ratios.min() < ratios.max()
    # one-pair signature of the reference
    k = 1
    assert overlap_ratio(frags[pairs[k, 0]], frags[pairs[k, 1]], trans[k], method) == \
        compute_overlap_ratio(frags[pairs[k, 0]], frags[pairs[k, 1]], trans[k], method)
