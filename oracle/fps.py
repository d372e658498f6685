"""Farthest point sampling restated in numpy (TEST ORACLE ONLY).

The reference calls pointnet2_ops `furthest_point_sample` (lib/layers.py:134-141; the package
is not vendored and its import is disabled in the source).  The
published algorithm, which this restatement fixes as the semantics (parity unpinned):
  idx[0] = 0; d[k] = +inf;
  for j = 1 .. m-1:  d[k] = min(d[k], |p_k - p_idx[j-1]|^2);  idx[j] = argmax_k d[k]
with the FIRST maximum on ties (numpy argmax) and no special-casing of points near the origin
(upstream skips |p|^2 <= 1e-3 as padding; DESIGN.md records the choice).
"""
import numpy as np


def furthest_point_sample(xyz, m):
    """xyz [n, 3] -> int64 [m] local indices."""
    p = np.asarray(xyz, dtype=np.float32)
    n = p.shape[0]
    if m > n:
        raise ValueError("m > n")
    idx = np.zeros(m, np.int64)
    d = np.full(n, np.inf, np.float32)
    last = 0
    for j in range(1, m):
        diff = p - p[last]
        d = np.minimum(d, (diff[:, 0] * diff[:, 0] + diff[:, 1] * diff[:, 1]) + diff[:, 2] * diff[:, 2])
        last = int(np.argmax(d))
        idx[j] = last
    return idx


def sample_fps(xyz, pts_list, targeted):
    """Sampler('fps') (lib/layers.py:128-141): num = min(targeted, min(pts)); per fragment FPS,
    indices offset to the fragment start -> [B, num] global rows."""
    num = min(targeted, min(pts_list))
    out, start = [], 0
    for n in pts_list:
        out.append(start + furthest_point_sample(xyz[start:start + n], num))
        start += n
    return np.stack(out)
