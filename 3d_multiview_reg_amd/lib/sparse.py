"""Sparse tensors on MI355X: the subset of MinkowskiEngine 0.4 that the FCGF
descriptor and the demo/extract pipelines use (ME.SparseTensor, the coordinate
manager with its strided coordinate sets and kernel maps,
ME.utils.sparse_quantize / sparse_collate), implemented on libmvreg_hip.so.

Coordinates are int32 [M, 4] = (batch, x, y, z) — batch FIRST (our convention;
ME 0.4 itself stored the batch index last).  Every coordinate set, hash table
and kernel map lives in HBM and is cached on the CoordinateManager shared by all
tensors of one forward pass.
"""
import ctypes
import os

import numpy as np
import torch

from lib import _native as N

# the ten 3^3 kernel maps of FCGF (lib/descriptor/fcgf.py; fcgf.py:118-227 of the reference): stride-1 stencils at
# tensor strides 1-8, the strided convs 1->2, 2->4, 4->8 and the transposed 8->4, 4->2, 2->1 (keyed by output stride)
FCGF_MAPS = (("s1", 1), ("s1", 2), ("s1", 4), ("s1", 8), ("down", 1), ("down", 2), ("down", 4),
             ("up", 4), ("up", 2), ("up", 1))
# MVR_SPATIAL_MAPS=1: 3^3 kernel maps visit their output rows in (fragment, Morton) order instead of the sets'
# first-occurrence order (identical maps).  Off by default: no gain on the same box (round 6, profiles/r06/
# ab_r6s1.txt: the coordinate work 2.58 ms per step in first-occurrence order vs 2.68 with the extra sort)
SPATIAL_MAPS = os.environ.get("MVR_SPATIAL_MAPS", "0") == "1"


class CoordinateManager:
    """Per-batch cache: stride -> coords / hash table; (kind, stride) -> neighbour table."""

    def __init__(self, coords, batch_size):
        self.B = int(batch_size)
        self.device = coords.device
        self.coords = {1: coords.contiguous()}
        self.tables = {}
        self.bricks = {}
        self.maps = {}
        self.orders = {}
        self.spatial = {}

    def coords_at(self, s):
        if s not in self.coords:
            prev = self.coords_at(s // 2)
            M = prev.shape[0]
            L = N.lib()
            ws = N.workspace(L.mvr_coords_downsample_workspace_bytes(M), self.device)
            out = torch.empty(M, 4, dtype=torch.int32, device=self.device)
            cnt = torch.empty(1 + self.B, dtype=torch.int64, device=self.device)
            N.check(L.mvr_coords_downsample(N.ptr(prev), M, self.B, s, N.ptr(ws), ws.numel(), N.ptr(out), N.ptr(cnt),
                                            N.stream()), "mvr_coords_downsample")
            n = int(cnt[0].item())
            self.coords[s] = out[:n]
        return self.coords[s]

    def table(self, s):
        if s not in self.tables:
            c = self.coords_at(s)
            L = N.lib()
            nb = L.mvr_hash_table_bytes(c.shape[0])
            t = torch.empty(nb, dtype=torch.uint8, device=self.device)
            N.check(L.mvr_hash_build_lattice(N.ptr(c), c.shape[0], s, N.ptr(t), nb, N.stream()),
                    "mvr_hash_build_lattice")
            self.tables[s] = t
        return self.tables[s]

    def brick_map(self, s):
        """4x4x4 brick map of the stride-s set (cells = coordinates / s; csrc/sparse.hip): the neighbourhood
        structure of the 3^3 kernel maps and of conv1's 7^3 stencil."""
        if s not in self.bricks:
            c = self.coords_at(s)
            L = N.lib()
            nb = L.mvr_brick_map_bytes(c.shape[0])
            t = torch.empty(nb, dtype=torch.uint8, device=self.device)
            N.check(L.mvr_brick_map_build_stride(N.ptr(c), c.shape[0], s, N.ptr(t), nb, N.stream()),
                    "mvr_brick_map_build_stride")
            self.bricks[s] = t
        return self.bricks[s]

    def spatial_orders(self, strides=(1, 2, 4, 8)):
        """(fragment, Morton code of coordinates / stride) order of each level's rows, all levels in ONE radix sort
        (mvr_kernel_map_orders without neighbour tables): the order the kernel maps visit their output rows in"""
        todo = [s for s in strides if s not in self.spatial]
        if not todo:
            return
        cs = [self.coords_at(s) for s in todo]
        Mo = [int(c.shape[0]) for c in cs]
        total, n = sum(Mo), len(todo)
        L = N.lib()
        ws = N.workspace(L.mvr_kernel_map_orders_bytes(total), self.device)
        perm = torch.empty(max(total, 1), dtype=torch.int32, device=self.device)
        vp = ctypes.c_void_p
        N.check(L.mvr_kernel_map_orders(n, None, (vp * n)(*[c.data_ptr() for c in cs]), (ctypes.c_int * n)(*todo),
                                        (ctypes.c_int64 * n)(*Mo), 0, N.ptr(perm), N.ptr(ws), ws.numel(), N.stream()),
                "mvr_kernel_map_orders (coordinates)")
        o = 0
        for s, m in zip(todo, Mo):
            self.spatial[s] = perm[o:o + m]
            o += m

    def kernel_map(self, kind, s, ks=3):
        """kind 's1': ks^3 stencil within stride s; 'down': stride s -> 2s; 'up': 2s -> s (transposed), resolved
        over the input level's lattice coordinate table (3^3 maps: output rows visited in spatial order)."""
        key = (kind, s, ks)
        if key not in self.maps:
            if kind == "s1":
                out_s, tab, tr = s, self.table(s), 0
            elif kind == "down":
                out_s, tab, tr = 2 * s, self.table(s), 0
            elif kind == "up":
                out_s, tab, tr = s, self.table(2 * s), 1
            else:
                raise ValueError(kind)
            out_c = self.coords_at(out_s)
            K = ks ** 3
            nbr = torch.empty(out_c.shape[0], K, dtype=torch.int32, device=self.device)
            L = N.lib()
            if ks == 3 and kind == "s1" and not SPATIAL_MAPS:
                # a set onto itself: half the offsets probed, each hit writes its mirror entry too
                N.check(L.mvr_kernel_map_sym(N.ptr(out_c), out_c.shape[0], N.ptr(tab), tab.numel(), s, N.ptr(nbr),
                                             N.stream()), "mvr_kernel_map_sym")
            elif ks == 3 and kind == "up" and not SPATIAL_MAPS:
                # the transposed conv's map is the transpose of the strided conv's map between the same two sets
                down = self.kernel_map("down", s, ks)
                N.check(L.mvr_kernel_map_transpose(N.ptr(down), down.shape[0], K, N.ptr(nbr), out_c.shape[0],
                                                   N.stream()), "mvr_kernel_map_transpose")
            else:
                order = None
                if ks == 3 and SPATIAL_MAPS:
                    self.spatial_orders()
                    order = self.spatial[out_s]
                N.check(L.mvr_kernel_map_x(N.ptr(out_c), out_c.shape[0], N.ptr(tab), tab.numel(), ks, s, tr,
                                           N.ptr(nbr), N.ptr(order), N.stream()), "mvr_kernel_map_x")
            self.maps[key] = nbr
        return self.maps[key]

    def _order_args(self, kind, s, ks):
        nbr = self.kernel_map(kind, s, ks)
        step = 2 * s if kind == "down" else s
        return nbr, self.coords_at(step), step

    def kernel_map_order(self, kind, s, ks=3):
        """Rows of kernel_map(kind, s) sorted by their active-offset mask, then fragment and Morton code of their
        coordinates (tiling order of mvr_spconv)."""
        key = (kind, s, ks)
        if key not in self.orders:
            nbr, out_c, step = self._order_args(kind, s, ks)
            L = N.lib()
            ws = N.workspace(L.mvr_kernel_map_order_bytes(nbr.shape[0]), self.device)
            perm = torch.empty(nbr.shape[0], dtype=torch.int32, device=self.device)
            N.check(L.mvr_kernel_map_order(N.ptr(nbr), N.ptr(out_c), step, nbr.shape[0], nbr.shape[1], N.ptr(perm),
                                           N.ptr(ws), ws.numel(), N.stream()), "mvr_kernel_map_order")
            self.orders[key] = perm
        return self.orders[key]

    def prepare_orders(self, specs=FCGF_MAPS, ks=3):
        """The kernel maps of `specs` ((kind, stride) pairs) and all their row orders in ONE sort
        (mvr_kernel_map_orders: the map index in the top key bits; the same orders as kernel_map_order one by one,
        with one histogram and eight digit passes for all of them instead of per map)."""
        todo = [(k, s) for k, s in specs if (k, s, ks) not in self.orders]
        if not todo:
            return
        args = [self._order_args(k, s, ks) for k, s in todo]
        n = len(args)
        Mo = [int(a[0].shape[0]) for a in args]
        total = sum(Mo)
        L = N.lib()
        ws = N.workspace(L.mvr_kernel_map_orders_bytes(total), self.device)
        perm = torch.empty(max(total, 1), dtype=torch.int32, device=self.device)
        vp = ctypes.c_void_p
        nbr_a = (vp * n)(*[a[0].data_ptr() for a in args])
        crd_a = (vp * n)(*[a[1].data_ptr() for a in args])
        stp_a = (ctypes.c_int * n)(*[a[2] for a in args])
        mo_a = (ctypes.c_int64 * n)(*Mo)
        N.check(L.mvr_kernel_map_orders(n, nbr_a, crd_a, stp_a, mo_a, ks ** 3, N.ptr(perm), N.ptr(ws), ws.numel(),
                                        N.stream()), "mvr_kernel_map_orders")
        o = 0
        for (k, s), m in zip(todo, Mo):
            self.orders[(k, s, ks)] = perm[o:o + m]
            o += m


class SparseTensor:
    """ME.SparseTensor(feats, coords=...) / (feats, coords_key=..., coords_manager=...)."""

    def __init__(self, feats, coords=None, coords_key=None, coords_manager=None, tensor_stride=1, batch_size=None):
        self.F = feats
        self.tensor_stride = tensor_stride
        if coords_manager is not None:
            self.coords_man = coords_manager
            self.coords_key = coords_key if coords_key is not None else tensor_stride
        else:
            if coords is None:
                raise ValueError("SparseTensor needs coords or a coords_manager")
            c = torch.as_tensor(coords).to(torch.int32)
            # batch_size (when the caller knows it, e.g. len(pts_list)) spares a device sync
            B = int(batch_size) if batch_size is not None else (int(c[:, 0].max().item()) + 1 if c.numel() else 1)
            self._pending = (c, B)
            self.coords_man = None
            self.coords_key = 1

    def to(self, device):
        self.F = self.F.to(device)
        if self.coords_man is None:
            c, B = self._pending
            self.coords_man = CoordinateManager(c.to(device).contiguous(), B)
        return self

    @property
    def C(self):
        return self.coords_man.coords_at(self.coords_key)


def voxelize(points_list, voxel_size, device, distinct_hint=None):
    """Batched sparse_quantize of raw fragments (scripts/pairwise_demo.py:74-96).
    points_list: list of float arrays/tensors [n_b, 3].  Returns (coords int32 [M,4],
    sel int64 [M] (global point index), counts list, xyz_down float32 [M,3]).
    float64 inputs (all of them) are floored as they are (mvr_voxelize_f64: the reference's np.floor on Open3D's
    float64 points); anything else is read as float32."""
    if points_list and all(p.dtype == torch.float64 if torch.is_tensor(p) else np.asarray(p).dtype == np.float64
                           for p in points_list):
        return _voxelize_f64(points_list, voxel_size, device)
    pts = [torch.as_tensor(np.asarray(p, dtype=np.float32)) if not torch.is_tensor(p) else p.float() for p in points_list]
    B = len(pts)
    n = [int(p.shape[0]) for p in pts]
    xyz = _adjacent_views(pts, device)
    if xyz is None:
        xyz = torch.cat(pts, 0).to(device).contiguous()
    off = torch.tensor(np.concatenate([[0], np.cumsum(n)]), dtype=torch.int64).pin_memory().to(device, non_blocking=True)
    total = int(sum(n))
    L = N.lib()
    coords = torch.empty(total, 4, dtype=torch.int32, device=device)
    sel = torch.empty(total, dtype=torch.int64, device=device)
    cnt = torch.empty(2 + B, dtype=torch.int64, device=device)
    dev_key = device.index if device.index is not None else torch.cuda.current_device()
    hint = _VOX_HINT.get(dev_key) if distinct_hint is None else distinct_hint
    c = None
    if hint:   # hash table sized for the expected voxel count; a key that finds no slot -> full-size re-run
        ws = N.workspace(L.mvr_voxelize_hint_workspace_bytes(total, int(hint)), device)
        N.check(L.mvr_voxelize_hint(N.ptr(xyz), N.ptr(off), B, total, float(voxel_size), int(hint), N.ptr(ws),
                                    ws.numel(), N.ptr(coords), N.ptr(sel), N.ptr(cnt), N.stream()), "mvr_voxelize_hint")
        c = cnt.cpu().numpy()
        if c[1 + B]:
            c = None
    if c is None:
        ws = N.workspace(L.mvr_voxelize_workspace_bytes(total), device)
        N.check(L.mvr_voxelize(N.ptr(xyz), N.ptr(off), B, total, float(voxel_size), N.ptr(ws), ws.numel(),
                               N.ptr(coords), N.ptr(sel), N.ptr(cnt), N.stream()), "mvr_voxelize")
        c = cnt.cpu().numpy()
    M = int(c[0])
    _VOX_HINT[dev_key] = max(3 * M // 2, 1024)   # the next call's table: this cloud's voxels + 50 %
    coords, sel = coords[:M], sel[:M]
    xyz_down = torch.empty(M, 3, device=device)
    N.check(L.mvr_gather_rows(N.ptr(xyz), 3, N.ptr(sel), M, N.ptr(xyz_down), N.stream()), "mvr_gather_rows")
    return coords, sel, [int(v) for v in c[1:1 + B]], xyz_down


def _voxelize_f64(points_list, voxel_size, device):
    """voxelize() of float64 fragments (mvr_voxelize_f64), same outputs; xyz_down rounded to float32 after the
    gather (the reference's pcd0 is float32, scripts/pairwise_demo.py:92)"""
    pts = [torch.as_tensor(np.asarray(p)) if not torch.is_tensor(p) else p for p in points_list]
    B = len(pts)
    n = [int(p.shape[0]) for p in pts]
    xyz = torch.cat([p.reshape(-1, 3) for p in pts], 0).to(device).contiguous()
    off = torch.tensor(np.concatenate([[0], np.cumsum(n)]), dtype=torch.int64).to(device)
    total = int(sum(n))
    L = N.lib()
    coords = torch.empty(total, 4, dtype=torch.int32, device=device)
    sel = torch.empty(total, dtype=torch.int64, device=device)
    cnt = torch.empty(1 + B, dtype=torch.int64, device=device)
    ws = N.workspace(L.mvr_voxelize_workspace_bytes(total), device)
    N.check(L.mvr_voxelize_f64(N.ptr(xyz), N.ptr(off), B, total, float(voxel_size), N.ptr(ws), ws.numel(),
                               N.ptr(coords), N.ptr(sel), N.ptr(cnt), N.stream()), "mvr_voxelize_f64")
    c = cnt.cpu().numpy()
    M = int(c[0])
    coords, sel = coords[:M], sel[:M]
    x32 = xyz.float()
    xyz_down = torch.empty(M, 3, device=device)
    N.check(L.mvr_gather_rows(N.ptr(x32), 3, N.ptr(sel), M, N.ptr(xyz_down), N.stream()), "mvr_gather_rows")
    return coords, sel, [int(v) for v in c[1:1 + B]], xyz_down


def fragment_views(points_list, device):
    """The fragments copied once into ONE contiguous device buffer, returned as views of it: voxelize() then
    reads them in place (no per-call concatenation of the raw points)."""
    pts = [torch.as_tensor(np.asarray(p, dtype=np.float32)) if not torch.is_tensor(p) else p.float() for p in points_list]
    buf = torch.cat([p.reshape(-1, 3).to(device) for p in pts], 0).contiguous()
    views, o = [], 0
    for p in pts:
        views.append(buf[o:o + p.shape[0]])
        o += p.shape[0]
    return views


def _adjacent_views(pts, device):
    """the [sum n, 3] tensor the fragments already form when they are consecutive row ranges of one contiguous
    buffer on `device` (fragment_views), else None"""
    if not pts:
        return None
    dev = torch.device(device)
    first = pts[0]
    if first.device.type != dev.type or (dev.index is not None and first.device.index != dev.index):
        return None
    ptr = first.data_ptr()
    base = first.untyped_storage().data_ptr()
    for p in pts:
        # consecutive in memory is not enough: separately allocated tensors can sit side by side in the caching
        # allocator, and set_() on the first one's (too small) storage would then resize it and leave the rest
        # uninitialised — every fragment must be a view of the SAME storage
        if p.device != first.device or p.dim() != 2 or p.shape[1] != 3 or p.dtype != torch.float32 or \
                not p.is_contiguous() or p.data_ptr() != ptr or p.untyped_storage().data_ptr() != base:
            return None
        ptr += p.numel() * 4
    total = sum(int(p.shape[0]) for p in pts)
    if (first.storage_offset() + total * 3) * 4 > first.untyped_storage().nbytes():
        return None
    return first.new_empty(0).set_(first.untyped_storage(), first.storage_offset(), (total, 3), (3, 1))


_VOX_HINT = {}   # per device: voxel-count estimate for the next voxelize() table (the last call's count + 50 %)
