"""Farthest point sampling on the GPU (replaces pointnet2_ops.furthest_point_sample as used by
lib/layers.py:134-141; semantics fixed in oracle/fps.py, csrc/fps.hip)."""
import numpy as np
import torch

from lib import _native as N


def furthest_point_sample(input_C, pts_list, num_points):
    """input_C [sum n, 3] (fragments back to back), pts_list [B] -> int64 [B, num_points] global rows
    (seed = first point of each fragment)."""
    N.require_hip(input_C)
    pts = np.asarray([int(p) for p in pts_list], dtype=np.int64)
    off = np.concatenate([[0], np.cumsum(pts)]).astype(np.int64)
    xyz = input_C.float().contiguous()
    off_dev = torch.from_numpy(off).to(xyz.device)
    out = torch.empty(len(pts), int(num_points), dtype=torch.int64, device=xyz.device)
    N.check(N.lib().mvr_fps(N.ptr(xyz), N.ptr(off_dev), off.ctypes.data, len(pts), int(num_points), N.ptr(out),
                            N.stream()), "mvr_fps")
    return out
