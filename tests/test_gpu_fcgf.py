"""FCGF sparse-voxel path on the GPU vs the numpy oracle (oracle/fcgf.py).
MinkowskiEngine cannot run here, so these comparisons pin our HIP kernels to
the oracle's restatement of the ME 0.4 conventions ('parity unpinned' w.r.t.
ME itself)."""
import numpy as np
import pytest

from synth import synth_scene_fragments, synth_state

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def frags():
    f, _ = synth_scene_fragments(3, seed=5, n_pts=60000)
    return f


def test_voxelize_matches_oracle(gpu, frags):
    from lib.sparse import voxelize
    from oracle.fcgf import voxelize as ovox
    c, sel, counts, xyz = voxelize(frags, 0.025, gpu)
    oc, osel, ocnt = ovox(frags, 0.025)
    assert counts == list(ocnt)
    np.testing.assert_array_equal(c.cpu().numpy(), oc)
    np.testing.assert_array_equal(sel.cpu().numpy(), osel)
    np.testing.assert_array_equal(xyz.cpu().numpy(), np.concatenate(frags)[osel])


def test_voxelize_float64_points_floored_as_given(gpu):
    """float64 clouds (Open3D's points in the reference's scripts/utils.py:108-109 extract_features) are floored
    in float64 as they are (mvr_voxelize_f64): points just below a voxel boundary, whose float32 rounding would
    land on or past it, keep the lower voxel — the oracle's np.floor(xyz / voxel) on the float64 array — and
    scripts.utils.extract_features keeps the float64 points it was given"""
    import torch
    from lib.sparse import voxelize
    from oracle.fcgf import voxelize as ovox
    rng = np.random.default_rng(3)
    k = rng.integers(-200, 200, (4000, 3))
    x = k * 0.025 - rng.uniform(1e-12, 1e-9, (4000, 3))          # just below the boundary k * 0.025
    x = np.concatenate([x, rng.uniform(-3, 3, (2000, 3))])
    oc, osel, ocnt = ovox([x], 0.025)
    c, sel, counts, xyz = voxelize([x], 0.025, gpu)
    assert counts == list(ocnt)
    np.testing.assert_array_equal(c.cpu().numpy(), oc)
    np.testing.assert_array_equal(sel.cpu().numpy(), osel)
    np.testing.assert_array_equal(xyz.cpu().numpy(), x[osel].astype(np.float32))
    # the test has teeth: the float32-rounded cloud gives other voxels
    c32, _, _ = ovox([x.astype(np.float32)], 0.025)
    assert len(c32) != len(oc) or not np.array_equal(c32, oc)
    # torch float64 on the device: the same
    c2, sel2, _, _ = voxelize([torch.from_numpy(x).to(gpu)], 0.025, gpu)
    np.testing.assert_array_equal(sel2.cpu().numpy(), osel)


@pytest.mark.parametrize("hint", [None, 1000, 10 ** 6, "exact"])
def test_voxelize_hint_sized_table_matches_oracle(gpu, frags, hint):
    """mvr_voxelize_hint: the hash table sized for the expected voxel count (lib.sparse keeps the last
    count + 50 %); a hint far too small overflows the bounded probing and re-runs at full size; every
    hint gives the oracle's voxels bit for bit."""
    from lib import sparse
    from oracle.fcgf import voxelize as ovox
    oc, osel, ocnt = ovox(frags, 0.025)
    h = len(oc) if hint == "exact" else hint
    sparse._VOX_HINT.clear()
    c, sel, counts, _ = sparse.voxelize(frags, 0.025, gpu, distinct_hint=h)
    assert counts == list(ocnt)
    np.testing.assert_array_equal(c.cpu().numpy(), oc)
    np.testing.assert_array_equal(sel.cpu().numpy(), osel)
    # the next call without an explicit hint uses the recorded one
    c2, sel2, counts2, _ = sparse.voxelize(frags, 0.025, gpu)
    assert counts2 == list(ocnt)
    np.testing.assert_array_equal(sel2.cpu().numpy(), osel)


@pytest.mark.parametrize("bricks", [False, True])
def test_strided_sets_and_kernel_maps_match_oracle(gpu, frags, bricks, monkeypatch):
    """every level's coordinate set and the 3^3 kernel maps (over the coordinate tables, and over brick maps:
    mvr_kernel_map_bricks) equal the oracle's"""
    import lib.sparse
    monkeypatch.setattr(lib.sparse, "BRICK_MAPS", bricks)
    from lib.sparse import voxelize, CoordinateManager
    from oracle.fcgf import Levels
    c, _, counts, _ = voxelize(frags, 0.025, gpu)
    cm = CoordinateManager(c, len(frags))
    lv = Levels(c.cpu().numpy())
    for l, s in enumerate((1, 2, 4, 8)):
        np.testing.assert_array_equal(cm.coords_at(s).cpu().numpy(), lv.coords[l])
    for kind, s in (("s1", 1), ("s1", 4), ("down", 1), ("down", 4), ("up", 1), ("up", 4)):
        l = {1: 0, 2: 1, 4: 2, 8: 3}[s]
        np.testing.assert_array_equal(cm.kernel_map(kind, s).cpu().numpy(), lv.nbr(kind, l), err_msg=kind + str(s))


def test_kernel_map_k7_property(gpu, frags):
    """every voxel finds itself at the centre offset; the map is symmetric"""
    from lib.sparse import voxelize, CoordinateManager
    c, _, _, _ = voxelize(frags[:1], 0.025, gpu)
    cm = CoordinateManager(c, 1)
    nbr = cm.kernel_map("s1", 1, ks=7).cpu().numpy()
    K = 343
    assert np.array_equal(nbr[:, K // 2], np.arange(len(nbr)))
    o, k = np.nonzero(nbr >= 0)
    assert np.array_equal(nbr[nbr[o, k], K - 1 - k], o)


@pytest.mark.parametrize("stride", [1, 2, 4])
def test_lattice_table_kernel_maps_dense_and_sparse(gpu, stride):
    """mvr_hash_build_lattice (cells of 8 voxels share a bucket): dense blocks fill whole buckets so inserts overflow
    into the next ones, beside scattered voxels and two batches; the kernel maps (s1, transposed) equal the hashed
    table's (mvr_hash_build) and a brute-force dictionary lookup"""
    import torch
    from lib import _native as N
    L = N.lib()
    rng = np.random.default_rng(3 + stride)
    pts = set()
    for b in range(2):
        g = np.arange(-6, 6) * stride
        for x in g:
            for y in g:
                for z in g[:4]:
                    pts.add((b, int(x), int(y), int(z)))
        for _ in range(3000):
            pts.add((b,) + tuple(int(v) * stride for v in rng.integers(-200, 200, 3)))
    coords = np.array(sorted(pts, key=lambda p: rng.random()), dtype=np.int32)
    M = len(coords)
    cd = torch.from_numpy(coords).to(gpu)
    nb = L.mvr_hash_table_bytes(M)
    tl = torch.empty(nb, dtype=torch.uint8, device=gpu)
    th = torch.empty(nb, dtype=torch.uint8, device=gpu)
    N.check(L.mvr_hash_build_lattice(N.ptr(cd), M, stride, N.ptr(tl), nb, N.stream()), "lattice")
    N.check(L.mvr_hash_build(N.ptr(cd), M, N.ptr(th), nb, N.stream()), "hashed")
    assert L.mvr_hash_build_lattice(N.ptr(cd), M, 3, N.ptr(tl), nb, N.stream()) != 0   # not a power of two
    index = {tuple(r): i for i, r in enumerate(coords.tolist())}
    for tr in (0, 1):
        maps = []
        for t in (tl, th):
            nbr = torch.empty(M, 27, dtype=torch.int32, device=gpu)
            N.check(L.mvr_kernel_map(N.ptr(cd), M, N.ptr(t), nb, 3, stride, tr, N.ptr(nbr), N.stream()), "map")
            maps.append(nbr.cpu().numpy())
        np.testing.assert_array_equal(maps[0], maps[1])
        sg = -1 if tr else 1
        ref = np.full((M, 27), -1, np.int32)
        for o, (b, x, y, z) in enumerate(coords.tolist()):
            for k in range(27):
                dx, dy, dz = k % 3 - 1, (k // 3) % 3 - 1, k // 9 - 1
                ref[o, k] = index.get((b, x + sg * dx * stride, y + sg * dy * stride, z + sg * dz * stride), -1)
        np.testing.assert_array_equal(maps[0], ref)
        # the brick-map kernel map over the same set (mvr_kernel_map_bricks): the same table
        nbb = L.mvr_brick_map_bytes(M)
        br = torch.empty(nbb, dtype=torch.uint8, device=gpu)
        N.check(L.mvr_brick_map_build_stride(N.ptr(cd), M, stride, N.ptr(br), nbb, N.stream()), "bricks")
        nbr = torch.empty(M, 27, dtype=torch.int32, device=gpu)
        N.check(L.mvr_kernel_map_bricks(N.ptr(cd), M, stride, N.ptr(br), M, nbb, stride, stride, tr, N.ptr(nbr), None,
                                        N.stream()), "brick map")
        np.testing.assert_array_equal(nbr.cpu().numpy(), ref)


def test_brick_kernel_maps_equal_table_maps(gpu, frags, monkeypatch):
    """All ten 3^3 kernel maps of FCGF (s1 at strides 1-8, down 1-4, up 1-4) over the input level's brick map
    (mvr_kernel_map_bricks) equal the maps over the level's lattice coordinate table (mvr_kernel_map), and the row
    orders from the brick kernel's keys (mvr_kernel_map_order_keys) equal mvr_kernel_map_order's"""
    import torch
    import lib.sparse
    from lib import _native as N
    from lib.sparse import voxelize, CoordinateManager
    monkeypatch.setattr(lib.sparse, "BRICK_MAPS", True)
    L = N.lib()
    c, _, counts, _ = voxelize(frags, 0.025, gpu)
    cm = CoordinateManager(c, len(counts))
    maps = [("s1", s) for s in (1, 2, 4, 8)] + [(k, s) for k in ("down", "up") for s in (1, 2, 4)]
    for kind, s in maps:
        nbr_b = cm.kernel_map(kind, s)
        perm_b = cm.kernel_map_order(kind, s)
        out_s, in_s, tr = {"s1": (s, s, 0), "down": (2 * s, s, 0), "up": (s, 2 * s, 1)}[kind]
        out_c, in_c = cm.coords_at(out_s), cm.coords_at(in_s)
        nb = L.mvr_hash_table_bytes(in_c.shape[0])
        tab = torch.empty(nb, dtype=torch.uint8, device=gpu)
        N.check(L.mvr_hash_build_lattice(N.ptr(in_c), in_c.shape[0], in_s, N.ptr(tab), nb, N.stream()), "table")
        nbr_t = torch.empty_like(nbr_b)
        N.check(L.mvr_kernel_map(N.ptr(out_c), out_c.shape[0], N.ptr(tab), nb, 3, s, tr, N.ptr(nbr_t), N.stream()),
                "map")
        assert torch.equal(nbr_b, nbr_t), (kind, s)
        ws = N.workspace(L.mvr_kernel_map_order_bytes(nbr_t.shape[0]), gpu)
        perm_t = torch.empty_like(perm_b)
        N.check(L.mvr_kernel_map_order(N.ptr(nbr_t), N.ptr(out_c), out_s, nbr_t.shape[0], 27, N.ptr(perm_t), N.ptr(ws),
                                       ws.numel(), N.stream()), "order")
        assert torch.equal(perm_b, perm_t), (kind, s)


def test_fcgf_forward_matches_oracle(gpu, frags):
    """split-bf16 sparse convs on mvr_spconv_wimage images; the oracle is our restatement of ME's sparse conv
    (parity unpinned: ME is absent)"""
    import torch
    from lib.descriptor.fcgf import FCGFNet
    from lib.sparse import voxelize, SparseTensor
    from oracle.fcgf import fcgf_forward
    net = FCGFNet()
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    st = synth_state(shapes, seed=3)
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    net = net.to(gpu).eval()
    c, _, _, _ = voxelize(frags, 0.025, gpu)
    F = torch.ones(c.shape[0], 1, device=gpu)
    with torch.no_grad():
        out = net(SparseTensor(F, coords=c).to(gpu)).F.cpu().numpy()
    ref, _ = fcgf_forward(st, c.cpu().numpy(), np.ones((c.shape[0], 1), np.float32))
    assert out.shape == ref.shape == (c.shape[0], 32)
    np.testing.assert_allclose(np.linalg.norm(out, axis=1), 1.0, atol=1e-5)
    err = np.abs(out - ref).max()
    assert err < 2e-4, err


def test_kernel_map_order_mask_then_morton(gpu, frags):
    """mvr_kernel_map_order: perm is a permutation of the output rows, sorted by active-offset mask, then (with the
    output coordinates) by fragment and Morton code of coordinates / step, stably — the tiling order of the sparse
    convs (only the order changes: test_gpu_spconv checks results with and without it)"""
    from lib.sparse import voxelize, CoordinateManager
    c, _, counts, _ = voxelize(frags, 0.025, gpu)
    cm = CoordinateManager(c, len(counts))
    for kind, s in (("s1", 1), ("down", 1), ("up", 2), ("s1", 4)):
        nbr = cm.kernel_map(kind, s).cpu().numpy()
        perm = cm.kernel_map_order(kind, s).cpu().numpy()
        out_c = cm.coords_at(2 * s if kind == "down" else s).cpu().numpy().astype(np.int64)
        step = 2 * s if kind == "down" else s
        assert np.array_equal(np.sort(perm), np.arange(len(nbr)))
        mask = ((nbr >= 0).astype(np.int64) << np.arange(nbr.shape[1])).sum(1)

        def spread(v):
            v = v & 511
            out = np.zeros_like(v)
            for b in range(9):
                out |= ((v >> b) & 1) << (3 * b)
            return out
        q = out_c[:, 1:] // step
        lo = ((out_c[:, 0] & 31) << 27) | (spread(q[:, 0] & 511) << 2) | (spread(q[:, 1] & 511) << 1) | spread(q[:, 2] & 511)
        key = (mask << 32) | lo
        assert np.array_equal(perm, np.argsort(key, kind="stable"))


def test_brick_kernel_map_edge_cases(gpu):
    """mvr_kernel_map_bricks / mvr_brick_map_build_stride: an empty input set (every neighbour absent), an empty
    output set (no launch), negative coordinates across brick boundaries, a transposed map whose neighbours are off
    the coarse lattice for odd cells, and the argument checks"""
    import torch
    from lib import _native as N
    L = N.lib()
    # empty input set
    oc = torch.tensor([[0, 0, 0, 0], [0, -1, 5, -9]], dtype=torch.int32, device=gpu)
    nbb = L.mvr_brick_map_bytes(0)
    br = torch.empty(nbb, dtype=torch.uint8, device=gpu)
    N.check(L.mvr_brick_map_build_stride(N.ptr(oc), 0, 1, N.ptr(br), nbb, N.stream()), "empty bricks")
    nbr = torch.zeros(2, 27, dtype=torch.int32, device=gpu)
    N.check(L.mvr_kernel_map_bricks(N.ptr(oc), 2, 1, N.ptr(br), 0, nbb, 1, 1, 0, N.ptr(nbr), None, N.stream()), "map")
    assert (nbr.cpu().numpy() == -1).all()
    assert L.mvr_kernel_map_bricks(N.ptr(oc), 0, 1, N.ptr(br), 0, nbb, 1, 1, 0, N.ptr(nbr), None, N.stream()) == 0
    assert L.mvr_kernel_map_bricks(N.ptr(oc), 2, 1, N.ptr(br), 0, nbb, 3, 1, 0, N.ptr(nbr), None, N.stream()) != 0
    assert L.mvr_brick_map_build_stride(N.ptr(oc), 2, 6, N.ptr(br), L.mvr_brick_map_bytes(2), N.stream()) != 0
    # fine set around the origin (negative coordinates, brick boundaries at multiples of 4 cells), coarse set = the
    # stride-2 cells it covers; up map (coarse -> fine, transposed) and down map (fine -> coarse) vs brute force
    g = np.arange(-5, 5)
    fine = np.array([(b, x, y, z) for b in range(2) for x in g for y in g for z in (-1, 0, 3)], dtype=np.int32)
    coarse = np.unique(np.concatenate([fine[:, :1], np.floor_divide(fine[:, 1:], 2) * 2], 1), axis=0).astype(np.int32)
    idx = {s: {tuple(r): i for i, r in enumerate(c.tolist())} for s, c in ((1, fine), (2, coarse))}
    tf, tc = torch.from_numpy(fine).to(gpu), torch.from_numpy(coarse).to(gpu)
    bf, bc = (torch.empty(L.mvr_brick_map_bytes(len(c)), dtype=torch.uint8, device=gpu) for c in (fine, coarse))
    N.check(L.mvr_brick_map_build_stride(N.ptr(tf), len(fine), 1, N.ptr(bf), bf.numel(), N.stream()), "bf")
    N.check(L.mvr_brick_map_build_stride(N.ptr(tc), len(coarse), 2, N.ptr(bc), bc.numel(), N.stream()), "bc")
    for name, out, o_s, br_, in_s, tr, src in (("up", tf, 1, bc, 2, 1, coarse), ("down", tc, 2, bf, 1, 0, fine)):
        nb = torch.empty(out.shape[0], 27, dtype=torch.int32, device=gpu)
        N.check(L.mvr_kernel_map_bricks(N.ptr(out), out.shape[0], o_s, N.ptr(br_), len(src), br_.numel(), in_s, 1, tr,
                                        N.ptr(nb), None, N.stream()), name)
        ref = np.full((out.shape[0], 27), -1, np.int32)
        sg = -1 if tr else 1
        for o, (b, x, y, z) in enumerate(out.cpu().numpy().tolist()):
            for k in range(27):
                dx, dy, dz = k % 3 - 1, (k // 3) % 3 - 1, k // 9 - 1
                ref[o, k] = idx[in_s].get((b, x + sg * dx, y + sg * dy, z + sg * dz), -1)
        np.testing.assert_array_equal(nb.cpu().numpy(), ref, err_msg=name)


def test_fcgf_forward_independent_of_tiling_order(gpu, frags, monkeypatch):
    """The sparse convs' row order only decides which rows share a tile: every output row sums its active offsets in
    offset order whatever else its tile holds (inactive offsets add exact zeros), so FCGF's output is bit-identical
    over the table path (mask-then-Morton order), the brick path (the same order from the brick kernel's keys), the
    brick path with the spatial order for the s1 / strided maps (MVR_SPCONV_ORDER=spatial) and XCD-contiguous tiles."""
    import torch
    import lib.sparse
    from lib import _native as NV
    from lib.descriptor.fcgf import FCGFNet
    from lib.sparse import voxelize, SparseTensor
    net = FCGFNet()
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    st = synth_state(shapes, seed=4)
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    net = net.to(gpu).eval()
    c, _, _, _ = voxelize(frags, 0.025, gpu)
    F = torch.ones(c.shape[0], 1, device=gpu)
    outs = []
    L = NV.lib()
    for bricks, order, xcd in ((False, "mask", 0), (True, "mask", 0), (True, "spatial", 0), (True, "spatial", 1)):
        monkeypatch.setattr(lib.sparse, "BRICK_MAPS", bricks)
        monkeypatch.setattr(lib.sparse, "SPCONV_ORDER", order)
        prev = L.mvr_set_spconv_xcd(xcd)
        try:
            with torch.no_grad():
                outs.append(net(SparseTensor(F, coords=c).to(gpu)).F.clone())
        finally:
            L.mvr_set_spconv_xcd(prev)
    for i, o in enumerate(outs[1:], 1):
        assert torch.equal(outs[0], o), (i, (outs[0] - o).abs().max().item())
