"""Overlap gate of the pairwise benchmark on the GPU (replaces lib/utils.py:713-786
compute_overlap_ratio, called per pair at scripts/benchmark_pairwise_registration.py:219-220).

    ratio = max(#{p in pc_i : NN_dist(p, trans . pc_j) < r} / |pc_i|,
                #{q in pc_j : NN_dist(q, trans^-1 . pc_i) < r} / |pc_j|)

'FCGF' method (the benchmark default): both clouds are first reduced by Open3D's
VoxelDownSample(voxel_size) and r = 3 voxel_size; '3DMatch': raw points, r = 0.05.

`FragmentOverlap` downsamples and indexes the fragments of a scene once and then scores any
batch of (pair, transform) in one launch (csrc/overlap.hip); `overlap_ratio` keeps the
reference's one-pair signature.  Geometry is fp64 like the reference's numpy/sklearn path."""
import numpy as np
import torch

from lib import _native as N

R_3DMATCH = 0.05


def _radius(method, voxel_size):
    if method == "FCGF":
        return 3.0 * voxel_size
    if method == "3DMatch":
        return R_3DMATCH
    raise ValueError("Wrong overlap computation method was selected: %r" % (method,))


class FragmentOverlap(object):
    """Downsampled (method 'FCGF') or raw ('3DMatch') fragments of a scene with a radius index on the
    GPU.  xyz_list: list of [n_b, 3] arrays / tensors (any float dtype)."""

    def __init__(self, xyz_list, method="FCGF", voxel_size=0.025, device=None):
        N.require_hip()
        dev = device or torch.device("cuda", torch.cuda.current_device())
        self.method, self.voxel_size, self.r = method, float(voxel_size), _radius(method, voxel_size)
        L = N.lib()
        B = len(xyz_list)
        pts = [torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x) for x in xyz_list]
        n_raw = np.array([int(p.shape[0]) for p in pts], dtype=np.int64)
        off_raw = np.concatenate([[0], np.cumsum(n_raw)]).astype(np.int64)
        if method == "FCGF":
            xyz = torch.cat([p.reshape(-1, 3).to(dev, torch.float32) for p in pts]).contiguous()
            off_dev = torch.from_numpy(off_raw).to(dev)
            n = int(off_raw[-1])
            ws_b = L.mvr_voxel_centroids_workspace_bytes(n)
            ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)
            cent = torch.empty(max(n, 1), 3, dtype=torch.float64, device=dev)
            off = torch.empty(B + 1, dtype=torch.int64, device=dev)
            N.check(L.mvr_voxel_centroids(N.ptr(xyz), N.ptr(off_dev), B, n, self.voxel_size, N.ptr(ws), ws_b,
                                          N.ptr(cent), N.ptr(off), N.stream()), "mvr_voxel_centroids")
            self.off = off.cpu().numpy()
            self.xyz = cent[:int(self.off[-1])].contiguous()
        else:
            self.xyz = torch.cat([p.reshape(-1, 3).to(dev, torch.float64) for p in pts]).contiguous()
            self.off = off_raw
        self.B, self.M = B, int(self.off[-1])
        self.off_dev = torch.from_numpy(self.off).to(dev)
        self.max_points = int(np.max(np.diff(self.off))) if B else 0
        ib = L.mvr_radius_index_bytes(self.M)
        self.index = torch.empty(ib, dtype=torch.uint8, device=dev)
        N.check(L.mvr_radius_index_build(N.ptr(self.xyz), N.ptr(self.off_dev), B, self.M, self.r, N.ptr(self.index),
                                         ib, N.stream()), "mvr_radius_index_build")
        self.device = dev

    def counts(self, pairs, trans):
        """pairs [P, 2] fragment indices, trans [P, 4, 4] (the `trans` argument of the reference) ->
        int [P, 2] matched query points (pc_i side, pc_j side)."""
        pairs = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
        trans = np.asarray(trans, dtype=np.float64).reshape(-1, 4, 4)
        P = pairs.shape[0]
        T = np.empty((P, 2, 3, 4), np.float64)
        for k in range(P):
            T[k, 0] = np.linalg.inv(trans[k])[:3]   # pc_i mapped into the frame of pc_j
            T[k, 1] = trans[k][:3]                  # pc_j mapped into the frame of pc_i
        gp = torch.from_numpy(pairs).to(self.device)
        gT = torch.from_numpy(T).to(self.device)
        cnt = torch.empty(max(P, 1), 2, dtype=torch.int32, device=self.device)
        N.check(N.lib().mvr_radius_overlap_count(N.ptr(self.index), self.index.numel(), N.ptr(self.xyz),
                                                 N.ptr(self.off_dev), self.B, self.M, N.ptr(gp), N.ptr(gT), P,
                                                 self.max_points, self.r, N.ptr(cnt), N.stream()),
                "mvr_radius_overlap_count")
        return cnt[:P].cpu().numpy()

    def ratios(self, pairs, trans):
        """-> float64 [P]: max of the two overlap ratios (utils.py:779-786)."""
        pairs = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
        c = self.counts(pairs, trans).astype(np.float64)
        n = np.diff(self.off).astype(np.float64)
        return np.maximum(c[:, 0] / n[pairs[:, 0]], c[:, 1] / n[pairs[:, 1]])


def overlap_ratio(pc_i, pc_j, trans, method="3DMatch", voxel_size=0.025):
    """utils.py:713 compute_overlap_ratio(pc_i, pc_j, trans, method, voxel_size) for one pair."""
    fo = FragmentOverlap([pc_i, pc_j], method, voxel_size)
    return float(fo.ratios([[0, 1]], [trans])[0])
