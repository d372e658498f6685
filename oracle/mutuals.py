"""Coordinate-space nearest neighbour and the mutual-NN flag restated in numpy (TEST ORACLE ONLY).

knn1     <- /root/reference/lib/utils.py:274-299 knn_point(k=1): d = sum(-(pos1 - pos2)^2, -1) in fp32, summed
            left to right ((dx^2 + dy^2) + dz^2), nearest = first index of the minimum
mutuals  <- lib/utils.py:822-848 extract_mutuals: j = knn1(x1_soft_matches -> x2); flag = |x1 - x2m[j]|^2 < thr^2
            (thr^2 compared in fp32, as the reference's float32 tensor against a Python scalar)

Pinned by tests/golden/mutuals.npz, which the reference itself produced (tests/golden/make_golden.py)."""
import numpy as np


def _sq3(d):
    d = d.astype(np.float32)
    return (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]


def knn1(pos1, pos2, chunk=256):
    """pos1 [B, N, 3] targets, pos2 [B, M, 3] queries -> (dist [B, M] float32, idx [B, M] int64)."""
    pos1 = np.asarray(pos1, np.float32)
    pos2 = np.asarray(pos2, np.float32)
    B, M = pos2.shape[:2]
    dist = np.empty((B, M), np.float32)
    idx = np.empty((B, M), np.int64)
    for b in range(B):
        for q0 in range(0, M, chunk):
            d = _sq3(pos1[b][None, :, :] - pos2[b, q0:q0 + chunk, None, :])
            i = np.argmin(d, axis=1)
            idx[b, q0:q0 + chunk] = i
            dist[b, q0:q0 + chunk] = d[np.arange(d.shape[0]), i]
    return dist, idx


def mutuals(x1, x2, x1m, x2m, threshold=0.05):
    """-> (flags [B, N] float32, idx [B, N] int64)."""
    _, idx = knn1(x2, x1m)
    back = np.take_along_axis(np.asarray(x2m, np.float32), idx[..., None], axis=1)
    d = _sq3(np.asarray(x1, np.float32) - back)
    return (d < np.float32(threshold ** 2)).astype(np.float32), idx
