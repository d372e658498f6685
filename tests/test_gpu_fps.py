"""GPU farthest point sampling (csrc/fps.hip via lib.fps / Sampler('fps')) vs the numpy
restatement oracle/fps.py — indices bit-exact (parity unpinned: pointnet2_ops is not vendored)."""
import numpy as np
import pytest

from synth import synth_scene_fragments

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sizes,m", [([100, 257], 50), ([3000, 5000, 1024], 700), ([20000], 600), ([24000, 17000], 900),
                                    ([30000], 300), ([4096, 8192, 16384], 1000)])
def test_fps_matches_oracle(gpu, sizes, m):
    import torch
    from lib.fps import furthest_point_sample
    from oracle.fps import sample_fps
    r = np.random.RandomState(sum(sizes))
    xyz = np.concatenate([r.uniform(-2, 2, (n, 3)).astype(np.float32) for n in sizes])
    got = furthest_point_sample(torch.from_numpy(xyz).to(gpu), sizes, m).cpu().numpy()
    ref = sample_fps(xyz, sizes, m)
    np.testing.assert_array_equal(got, ref)


def test_sampler_fps_on_voxelised_fragments(gpu):
    import torch
    from lib.layers import Sampler
    from lib.sparse import voxelize
    from oracle.fps import sample_fps
    frags, _ = synth_scene_fragments(2, seed=3, n_pts=40000)
    coords, sel, counts, xyz = voxelize([torch.from_numpy(f) for f in frags], 0.025, gpu)
    F = torch.randn(xyz.shape[0], 32, device=gpu)
    sc, sf = Sampler("fps", 800)(xyz, F, torch.tensor(counts))
    idx = sample_fps(xyz.cpu().numpy(), counts, 800)
    np.testing.assert_array_equal(sc.cpu().numpy(), xyz.cpu().numpy()[idx])
    np.testing.assert_array_equal(sf.cpu().numpy(), F.cpu().numpy()[idx])


def test_fps_rejects_too_few_points(gpu):
    import torch
    from lib.fps import furthest_point_sample
    with pytest.raises(RuntimeError):
        furthest_point_sample(torch.zeros(10, 3, device=gpu), [10], 11)


def test_fps_ties_take_the_lowest_index(gpu):
    """exact distance ties (duplicated points, a lattice): the first maximum in fragment order wins, as numpy's
    argmax in the oracle"""
    import torch
    from lib.fps import furthest_point_sample
    from oracle.fps import sample_fps
    g = np.stack(np.meshgrid(*[np.arange(12, dtype=np.float32)] * 3, indexing="ij"), -1).reshape(-1, 3)
    xyz = np.concatenate([g, g[::-1], g[:500]])            # every point at least twice
    sizes = [len(xyz)]
    got = furthest_point_sample(torch.from_numpy(xyz).to(gpu), sizes, 700).cpu().numpy()
    np.testing.assert_array_equal(got, sample_fps(xyz, sizes, 700))
