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


def test_voxelize_partitioned_buckets(gpu):
    """mvr_voxelize_hint's partitioned dedup (workgroup = fragment x hash bucket, LDS table, the buckets of a fragment
    on one XCD): 11 fragments of unequal size (fragments past the first 8 take the second round of XCD slots) at
    hints giving 1, 2, 8 and 64 buckets per fragment; a hint too small for one LDS table and a coordinate outside the
    keys' 17-bit range both report overflow (counts_out[B + 1]) rather than wrong voxels"""
    import torch
    from lib import _native as N
    from lib import sparse
    from oracle.fcgf import voxelize as ovox
    fr, _ = synth_scene_fragments(11, seed=9, n_pts=30000)
    fr = [f[: 30000 - 2000 * i] for i, f in enumerate(fr)]
    oc, osel, ocnt = ovox(fr, 0.025)
    M = len(oc)
    for h in (M // 11, 2 * M, 8 * 4096 * 11, 64 * 4096 * 11):
        sparse._VOX_HINT.clear()
        c, sel, counts, _ = sparse.voxelize(fr, 0.025, gpu, distinct_hint=h)
        assert counts == list(ocnt), h
        np.testing.assert_array_equal(c.cpu().numpy(), oc)
        np.testing.assert_array_equal(sel.cpu().numpy(), osel)

    L = N.lib()

    def hint_call(pts, hint):
        xyz = torch.from_numpy(np.concatenate(pts).astype(np.float32)).to(gpu)
        off = torch.tensor(np.concatenate([[0], np.cumsum([len(p) for p in pts])]), dtype=torch.int64, device=gpu)
        n, B = xyz.shape[0], len(pts)
        ws = torch.empty(L.mvr_voxelize_hint_workspace_bytes(n, hint), dtype=torch.uint8, device=gpu)
        coords = torch.empty(n, 4, dtype=torch.int32, device=gpu)
        sel = torch.empty(n, dtype=torch.int64, device=gpu)
        cnt = torch.empty(2 + B, dtype=torch.int64, device=gpu)
        N.check(L.mvr_voxelize_hint(N.ptr(xyz), N.ptr(off), B, n, 0.025, hint, N.ptr(ws), ws.numel(), N.ptr(coords),
                                    N.ptr(sel), N.ptr(cnt), N.stream()), "mvr_voxelize_hint")
        return cnt.cpu().numpy()

    big = synth_scene_fragments(1, seed=2, n_pts=250000)[0][0]   # ~20 k voxels: more than one 8192-slot table
    assert hint_call([big], 1000)[2] != 0
    far = fr[0].copy()
    far[7] = (2000.0, 0.0, 0.0)                                   # 80 000 voxels from the origin
    cnt = hint_call([far], 10 ** 5)
    assert cnt[2] != 0
    assert hint_call([fr[0]], 10 ** 5)[2] == 0


def test_strided_sets_and_kernel_maps_match_oracle(gpu, frags):
    """every level's coordinate set and the 3^3 kernel maps equal the oracle's"""
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


def test_spatial_map_visit_order(gpu, frags, monkeypatch):
    """the 3^3 kernel maps visiting their output rows in (fragment, Morton) order (mvr_kernel_map_x + the
    coordinate-only mvr_kernel_map_orders) equal the maps built in row order, and each level's spatial order is the
    stable sort of those keys"""
    import torch
    import lib.sparse
    from lib.sparse import voxelize, CoordinateManager, FCGF_MAPS
    c, _, counts, _ = voxelize(frags, 0.025, gpu)
    monkeypatch.setattr(lib.sparse, "SPATIAL_MAPS", True)
    a = CoordinateManager(c, len(counts))
    monkeypatch.setattr(lib.sparse, "SPATIAL_MAPS", False)
    b = CoordinateManager(c, len(counts))
    for kind, s in FCGF_MAPS:
        monkeypatch.setattr(lib.sparse, "SPATIAL_MAPS", True)
        ma = a.kernel_map(kind, s)
        monkeypatch.setattr(lib.sparse, "SPATIAL_MAPS", False)
        assert torch.equal(ma, b.kernel_map(kind, s)), (kind, s)

    def spread(v):
        v = v & 511
        out = np.zeros_like(v)
        for bit in range(9):
            out |= ((v >> bit) & 1) << (3 * bit)
        return out
    for s in (1, 2, 4, 8):
        cs = a.coords_at(s).cpu().numpy().astype(np.int64)
        q = cs[:, 1:] // s
        lo = ((cs[:, 0] & 127) << 25) | (spread(q[:, 0] & 255) << 2) | (spread(q[:, 1] & 255) << 1) | spread(q[:, 2] & 255)
        np.testing.assert_array_equal(a.spatial[s].cpu().numpy(), np.argsort(lo, kind="stable"))


def test_batched_orders_equal_per_map_orders(gpu, frags):
    """CoordinateManager.prepare_orders (mvr_kernel_map_orders: all ten 3^3 maps of FCGF in ONE radix sort, the map
    index in the top key bits) gives every map exactly the order of mvr_kernel_map_order on that map alone; a
    subset of maps, and maps with no rows, too"""
    import torch
    from lib.sparse import voxelize, CoordinateManager, FCGF_MAPS
    c, _, counts, _ = voxelize(frags, 0.025, gpu)
    one, batch = CoordinateManager(c, len(counts)), CoordinateManager(c, len(counts))
    batch.prepare_orders()
    for kind, s in FCGF_MAPS:
        assert torch.equal(batch.kernel_map_order(kind, s), one.kernel_map_order(kind, s)), (kind, s)
    sub = CoordinateManager(c, len(counts))
    sub.prepare_orders((("up", 2), ("s1", 8)))
    for kind, s in (("up", 2), ("s1", 8)):
        assert torch.equal(sub.orders[(kind, s, 3)], one.kernel_map_order(kind, s)), (kind, s)
    # a map with no rows between two others
    from lib import _native as N
    L = N.lib()
    nbr = [one.kernel_map("s1", 4), one.kernel_map("s1", 8)]
    crd = [one.coords_at(4), one.coords_at(8)]
    empty = torch.empty(0, 27, dtype=torch.int32, device=gpu)
    import ctypes
    vp = ctypes.c_void_p
    Mo = [nbr[0].shape[0], 0, nbr[1].shape[0]]
    perm = torch.empty(sum(Mo), dtype=torch.int32, device=gpu)
    ws = N.workspace(L.mvr_kernel_map_orders_bytes(sum(Mo)), gpu)
    N.check(L.mvr_kernel_map_orders(3, (vp * 3)(nbr[0].data_ptr(), empty.data_ptr(), nbr[1].data_ptr()),
                                    (vp * 3)(crd[0].data_ptr(), crd[0].data_ptr(), crd[1].data_ptr()),
                                    (ctypes.c_int * 3)(4, 4, 8), (ctypes.c_int64 * 3)(*Mo), 27, N.ptr(perm), N.ptr(ws),
                                    ws.numel(), N.stream()), "orders")
    assert torch.equal(perm[:Mo[0]], one.kernel_map_order("s1", 4))
    assert torch.equal(perm[Mo[0]:], one.kernel_map_order("s1", 8))


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
        lo = ((out_c[:, 0] & 127) << 25) | (spread(q[:, 0] & 255) << 2) | (spread(q[:, 1] & 255) << 1) | spread(q[:, 2] & 255)
        key = (mask << 32) | lo
        assert np.array_equal(perm, np.argsort(key, kind="stable"))


def test_fcgf_forward_independent_of_tiling_order(gpu, frags, monkeypatch):
    """The sparse convs' row order only decides which rows share a tile: every output row sums its active offsets in
    offset order whatever else its tile holds (inactive offsets add exact zeros), so FCGF's output is bit-identical
    under the default order (mask, then fragment and Morton code), the identity order and a random permutation of
    every map's rows (injected in place of the kernel-map orders)."""
    import torch
    import lib.sparse
    from lib.descriptor.fcgf import FCGFNet
    from lib.sparse import voxelize, SparseTensor, CoordinateManager
    net = FCGFNet()
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    st = synth_state(shapes, seed=4)
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    net = net.to(gpu).eval()
    c, _, _, _ = voxelize(frags, 0.025, gpu)
    F = torch.ones(c.shape[0], 1, device=gpu)
    outs = []
    gen = torch.Generator(device="cpu").manual_seed(5)

    def injected(how):
        def order(self, kind, s, ks=3):
            n = self.kernel_map(kind, s, ks).shape[0]
            p = torch.arange(n, dtype=torch.int32) if how == "identity" else torch.randperm(n, generator=gen).int()
            return p.to(gpu)
        return order
    for how in ("default", "identity", "random"):
        if how != "default":
            monkeypatch.setattr(CoordinateManager, "prepare_orders", lambda self, *a, **k: None)
            monkeypatch.setattr(CoordinateManager, "kernel_map_order", injected(how))
        with torch.no_grad():
            outs.append(net(SparseTensor(F, coords=c).to(gpu)).F.clone())
    for i, o in enumerate(outs[1:], 1):
        assert torch.equal(outs[0], o), (i, (outs[0] - o).abs().max().item())


def test_empty_fragment_through_voxelize_and_orders(gpu, frags):
    """An empty fragment inside a batch, and a batch with no points at all, go through voxelize ->
    CoordinateManager (strided sets, lattice tables, kernel maps, prepare_orders): zero-element tensors hand the C ABI
    NULL pointers with zero counts, which every entry point accepts (include/mvreg.h conventions; round 5's
    mvr_radix_sort_pairs rejected them)."""
    import torch
    from lib.sparse import voxelize, CoordinateManager, FCGF_MAPS
    empty = np.zeros((0, 3), np.float32)
    c3, _, counts3, _ = voxelize([frags[0], empty, frags[2]], 0.025, gpu)
    c2, _, counts2, _ = voxelize([frags[0], frags[2]], 0.025, gpu)
    assert counts3 == [counts2[0], 0, counts2[1]]
    want = c2.cpu().numpy().copy()
    want[want[:, 0] == 1, 0] = 2                       # the third fragment keeps its batch index
    np.testing.assert_array_equal(c3.cpu().numpy(), want)
    a, b = CoordinateManager(c3, 3), CoordinateManager(c3, 3)
    a.prepare_orders()
    for kind, s in FCGF_MAPS:
        assert torch.equal(a.kernel_map_order(kind, s), b.kernel_map_order(kind, s)), (kind, s)
    # no points at all: every level, map and order is empty
    c0, sel0, counts0, xyz0 = voxelize([empty], 0.025, gpu)
    assert counts0 == [0] and c0.shape[0] == 0 and sel0.numel() == 0 and xyz0.shape[0] == 0
    z = CoordinateManager(c0, 1)
    z.prepare_orders()
    for kind, s in FCGF_MAPS:
        assert z.kernel_map(kind, s).shape[0] == 0 and z.orders[(kind, s, 3)].numel() == 0
    torch.cuda.synchronize()


@pytest.mark.parametrize("stride", [1, 2, 4])
def test_symmetric_and_transposed_kernel_maps(gpu, stride):
    """mvr_kernel_map_sym (a set onto itself: half the offsets probed, mirror entries written) equals mvr_kernel_map's
    full probe over lattice and hashed tables (dense blocks whose buckets overflow, scattered voxels, two batches), and
    mvr_kernel_map_transpose of the strided map fine -> coarse equals the transposed map coarse -> fine probed from
    the coarse table (FCGF's up maps from its down maps)"""
    import torch
    from lib import _native as N
    L = N.lib()
    rng = np.random.default_rng(11 + stride)
    pts = set()
    for b in range(2):
        g = np.arange(-5, 5) * stride
        for x in g:
            for y in g:
                for z in g[:3]:
                    pts.add((b, int(x), int(y), int(z)))
        for _ in range(2500):
            pts.add((b,) + tuple(int(v) * stride for v in rng.integers(-150, 150, 3)))
    fine = np.array(sorted(pts, key=lambda p: rng.random()), dtype=np.int32)
    coarse = np.unique(np.concatenate([fine[:, :1], (fine[:, 1:] // (2 * stride)) * (2 * stride)], 1), axis=0)
    coarse = coarse[rng.permutation(len(coarse))].astype(np.int32)
    Mf, Mc = len(fine), len(coarse)
    fd, cd = torch.from_numpy(fine).to(gpu), torch.from_numpy(coarse).to(gpu)

    def table(c, M, lat):
        t = torch.empty(L.mvr_hash_table_bytes(M), dtype=torch.uint8, device=gpu)
        if lat:
            N.check(L.mvr_hash_build_lattice(N.ptr(c), M, lat, N.ptr(t), t.numel(), N.stream()), "lattice")
        else:
            N.check(L.mvr_hash_build(N.ptr(c), M, N.ptr(t), t.numel(), N.stream()), "hashed")
        return t

    def kmap(oc, Mo, t, tr):
        nbr = torch.empty(Mo, 27, dtype=torch.int32, device=gpu)
        N.check(L.mvr_kernel_map(N.ptr(oc), Mo, N.ptr(t), t.numel(), 3, stride, tr, N.ptr(nbr), N.stream()), "map")
        return nbr
    for lat in (stride, 0):
        tf = table(fd, Mf, lat)
        sym = torch.empty(Mf, 27, dtype=torch.int32, device=gpu)
        N.check(L.mvr_kernel_map_sym(N.ptr(fd), Mf, N.ptr(tf), tf.numel(), stride, N.ptr(sym), N.stream()), "sym")
        assert torch.equal(sym, kmap(fd, Mf, tf, 0)), lat
    tf, tc = table(fd, Mf, stride), table(cd, Mc, 2 * stride)
    down = kmap(cd, Mc, tf, 0)                     # coarse rows, neighbours in the fine set
    up = kmap(fd, Mf, tc, 1)                       # fine rows, transposed neighbours in the coarse set
    assert int((down >= 0).sum()) > Mc             # the test has teeth
    upt = torch.empty(Mf, 27, dtype=torch.int32, device=gpu)
    N.check(L.mvr_kernel_map_transpose(N.ptr(down), Mc, 27, N.ptr(upt), Mf, N.stream()), "transpose")
    assert torch.equal(upt, up)
