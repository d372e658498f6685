"""CPU checks of the FCGF oracle's sparse-voxel conventions (oracle/fcgf.py)."""
import numpy as np

from oracle.fcgf import (voxelize, downsample, Table, kernel_map, offsets, sparse_conv, fcgf_state_shapes,
                         fcgf_forward, pack)
from synth import synth_scene_fragments, synth_state


def test_voxelize_first_occurrence_bruteforce():
    r = np.random.RandomState(0)
    xyz = [r.uniform(-0.3, 0.3, (2000, 3)), r.uniform(-0.2, 0.2, (1500, 3))]
    c, sel, cnt = voxelize(xyz, 0.05)
    seen, exp_c, exp_sel, base = {}, [], [], 0
    for b, p in enumerate(xyz):
        for i, q in enumerate(np.floor(p / 0.05).astype(int)):
            key = (b,) + tuple(q)
            if key not in seen:
                seen[key] = True
                exp_c.append(key)
                exp_sel.append(base + i)
        base += len(p)
    assert np.array_equal(c, np.asarray(exp_c))
    assert np.array_equal(sel, np.asarray(exp_sel))
    assert cnt.sum() == len(c)


def test_downsample_floor_negative_coords():
    c = np.array([[0, -1, -2, -3], [0, 1, 2, 3], [0, -2, -2, -4], [1, -1, -1, -1]], np.int32)
    d = downsample(c, 2)
    assert np.array_equal(d, np.array([[0, -2, -2, -4], [0, 0, 2, 2], [1, -2, -2, -2]]))


def test_sparse_conv_equals_dense_correlation():
    """fully occupied 6^3 block: the sparse conv is a dense 3-D cross-correlation with zero padding"""
    g = np.stack(np.meshgrid(np.arange(6), np.arange(6), np.arange(6), indexing="ij"), -1).reshape(-1, 3)
    c = np.concatenate([np.zeros((len(g), 1), int), g], 1)
    t = Table(c)
    nbr = kernel_map(c, t, 3, 1)
    r = np.random.RandomState(1)
    f = r.standard_normal((len(c), 2)).astype(np.float32)
    W = r.standard_normal((27, 2, 3)).astype(np.float32)
    out = sparse_conv(f, nbr, W)
    vol = np.zeros((8, 8, 8, 2), np.float32)
    vol[1:7, 1:7, 1:7] = f.reshape(6, 6, 6, 2)
    ref = np.zeros((6, 6, 6, 3), np.float32)
    for k, (dx, dy, dz) in enumerate(offsets(3)):
        ref += vol[1 + dx:7 + dx, 1 + dy:7 + dy, 1 + dz:7 + dz] @ W[k]
    np.testing.assert_allclose(out, ref.reshape(-1, 3), atol=1e-5)


def test_strided_and_transposed_maps_are_mirrors():
    frags, _ = synth_scene_fragments(1, seed=2, n_pts=20000)
    c, _, _ = voxelize(frags, 0.025)
    c2 = downsample(c, 2)
    down = kernel_map(c2, Table(c), 3, 1)                  # fine -> coarse
    up = kernel_map(c, Table(c2), 3, 1, transposed=True)  # coarse -> fine
    od, kd = np.nonzero(down >= 0)
    ou, ku = np.nonzero(up >= 0)
    pd = set(zip(od, down[od, kd], kd))        # (coarse o, fine i, k)
    pu = set(zip(up[ou, ku], ou, ku))          # (coarse input, fine output, k)
    assert pd == pu


def test_fcgf_forward_shapes_unit_norm():
    frags, _ = synth_scene_fragments(1, seed=3, n_pts=15000)
    c, _, _ = voxelize(frags, 0.025)
    st = synth_state(fcgf_state_shapes(), seed=1)
    F, lv = fcgf_forward(st, c, np.ones((len(c), 1), np.float32))
    assert F.shape == (len(c), 32)
    np.testing.assert_allclose(np.linalg.norm(F, axis=1), 1.0, atol=1e-5)
    assert len(lv.coords[3]) < len(lv.coords[2]) < len(lv.coords[1]) < len(c)


def test_pack_roundtrip_unique():
    r = np.random.RandomState(3)
    c = np.concatenate([r.randint(0, 40, (5000, 1)), r.randint(-60000, 60000, (5000, 3))], 1)
    k = pack(c)
    assert len(np.unique(k)) == len(np.unique(c, axis=0))


def test_demo_pair_voxel_counts():
    """The reference's demo pair (data/demo/pairwise/raw_data, committed under tests/golden/demo) voxelised at
    0.025 m by the oracle's sparse_quantize restatement: SURVEY §2.3's 18,977 / 19,082 voxels."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3d_multiview_reg_amd"))
    from lib.ply import read_ply_xyz
    from oracle.fcgf import voxelize
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "demo")
    pcs = [read_ply_xyz(os.path.join(d, "cloud_bin_%d.ply" % k)) for k in range(2)]
    _, _, counts = voxelize(pcs, 0.025)
    assert list(counts) == [18977, 19082]


def test_c_backend_equals_numpy_oracle():
    """oracle/csrc/sparse_conv.c (the CPU baseline's FCGF leg, C + OpenMP) against the numpy restatement: the same
    kernel maps (all kinds, 7^3 included) and features to fp32 rounding on a real fragment"""
    import os
    import subprocess
    from synth import synth_scene_fragments, synth_state
    from oracle.fcgf import voxelize, fcgf_forward, fcgf_state_shapes
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not os.path.exists(os.path.join(root, "oracle", "build", "libmvoracle.so")):
        subprocess.run(["make", "-C", os.path.join(root, "oracle")], check=True)
    frags, _ = synth_scene_fragments(2, seed=43, n_pts=40000)
    c, _, _ = voxelize(frags, 0.025)
    st = synth_state(fcgf_state_shapes(), seed=3)
    ones = np.ones((len(c), 1), np.float32)
    Fn, lvn = fcgf_forward(st, c, ones)
    Fc, lvc = fcgf_forward(st, c, ones, backend="c")
    for kind, l in (("s1", 0), ("s1", 3), ("down", 0), ("down", 2), ("up", 0), ("up", 2), ("k7", 0)):
        np.testing.assert_array_equal(lvn.nbr(kind, l), lvc.nbr(kind, l), err_msg="%s %d" % (kind, l))
    np.testing.assert_allclose(Fc, Fn, atol=2e-6)
