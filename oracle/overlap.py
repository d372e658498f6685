"""Overlap gate restated on the CPU (TEST ORACLE ONLY) — lib/utils.py:713-786 compute_overlap_ratio.

The NN part follows the reference's own calls (sklearn NearestNeighbors(n_neighbors=1,
algorithm='kd_tree'), fp64, strict `dist < r`).  The 'FCGF' method's open3d
`PointCloud.voxel_down_sample` (open3d is absent here; the reference pins no version, Open3D
0.8-0.9 by its `o3d.registration` API) is restated from the published algorithm
(VoxelDownSample): voxel index = floor((p - (min_bound - v/2)) / v) in fp64, output point = the
fp64 sum of the voxel's points in input order divided by their count (output order irrelevant
here).  Parity of that step is therefore unpinned."""
import numpy as np


def voxel_down_sample(xyz, voxel):
    p = np.asarray(xyz, dtype=np.float64).reshape(-1, 3)
    if p.shape[0] == 0:
        return p
    vmin = p.min(axis=0) - voxel * 0.5
    idx = np.floor((p - vmin) / voxel).astype(np.int64)
    _, inv = np.unique(idx, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    k = inv.max() + 1
    s = np.zeros((k, 3), np.float64)
    np.add.at(s, inv, p)            # unbuffered, in input order
    cnt = np.bincount(inv, minlength=k).astype(np.float64)
    return s / cnt[:, None]


def overlap_counts(pc_i, pc_j, trans, method="3DMatch", voxel_size=0.025):
    """-> (matching01, matching10, n_i, n_j) as in utils.py:734-776."""
    from sklearn.neighbors import NearestNeighbors
    trans = np.asarray(trans, dtype=np.float64)
    trans_inv = np.linalg.inv(trans)
    pc_i = np.asarray(pc_i, dtype=np.float64)
    pc_j = np.asarray(pc_j, dtype=np.float64)
    if method == "FCGF":
        pc_i, pc_j = voxel_down_sample(pc_i, voxel_size), voxel_down_sample(pc_j, voxel_size)
        r = 3 * voxel_size
    elif method == "3DMatch":
        r = 0.05
    else:
        raise ValueError(method)
    pc_i_t = (trans_inv[0:3, 0:3] @ pc_i.T + trans_inv[0:3, 3].reshape(-1, 1)).T
    pc_j_t = (trans[0:3, 0:3] @ pc_j.T + trans[0:3, 3].reshape(-1, 1)).T
    neigh = NearestNeighbors(n_neighbors=1, algorithm="kd_tree")
    neigh.fit(pc_j_t)
    d01, _ = neigh.kneighbors(pc_i, return_distance=True)
    neigh.fit(pc_i_t)
    d10, _ = neigh.kneighbors(pc_j, return_distance=True)
    return int((d01 < r).sum()), int((d10 < r).sum()), pc_i.shape[0], pc_j.shape[0]


def compute_overlap_ratio(pc_i, pc_j, trans, method="3DMatch", voxel_size=0.025):
    m01, m10, ni, nj = overlap_counts(pc_i, pc_j, trans, method, voxel_size)
    return max(m01 / ni, m10 / nj)
