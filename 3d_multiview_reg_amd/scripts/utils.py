"""scripts/utils.py of the reference (the helpers its scripts import) on the MI355X path.

  read_txt, ensure_dir          scripts/utils.py:16-41 (host file helpers)
  extract_features              scripts/utils.py:44-122: voxelise one cloud and run FCGF on it — here the
                                voxelisation is lib.sparse.voxelize (floor(x / voxel) in fp64 + first-occurrence dedup,
                                the ME.utils.sparse_quantize of :107-110) and the descriptor the HIP FCGFNet
  transform_point_cloud         scripts/utils.py:125-145 (numpy / torch)
  make_pairwise_eval_data_loader  scripts/utils.py:148-197 (in lib/data.py, re-exported under this path)
"""
import os

import numpy as np
import torch

from lib.data import make_pairwise_eval_data_loader  # noqa: F401


def read_txt(path):
    """scripts/utils.py:16-30: the stripped lines of a text file"""
    with open(path) as f:
        return [x.strip() for x in f.readlines()]


def ensure_dir(path):
    """scripts/utils.py:33-41"""
    if not os.path.exists(path):
        os.makedirs(path, mode=0o755)


def extract_features(model, xyz, rgb=None, normal=None, voxel_size=0.05, device=None, skip_check=False,
                     is_eval=True):
    """scripts/utils.py:44-122: (return_coords [m, 3] — the input points kept by the voxelisation, features
    [m, c]) of one point cloud xyz [n, 3].  Same checks, feature assembly (rgb - 0.5, normal / 2, or ones) and
    voxelisation (coords = floor(xyz / voxel_size), first occurrence kept) as the reference, on the device.
    The HIP FCGF takes a single input channel (every reference FCGF config: ones), so rgb / normal features raise."""
    if is_eval:
        model.eval()
    xyz = np.asarray(xyz)
    if not skip_check:
        assert xyz.shape[1] == 3
        n = xyz.shape[0]
        if rgb is not None:
            assert n == len(rgb)
            assert rgb.shape[1] == 3
            if np.any(rgb > 1):
                raise ValueError("Invalid color. Color must range from [0, 1]")
        if normal is not None:
            assert n == len(normal)
            assert normal.shape[1] == 3
            if np.any(normal > 1):
                raise ValueError("Invalid normal. Normal must range from [-1, 1]")
    if rgb is not None or normal is not None:
        raise NotImplementedError("FCGFNet on the HIP path takes one input channel (ones): rgb / normal inputs")
    if device is None:
        device = torch.device("cuda:0")
    from lib.sparse import SparseTensor, voxelize
    # floor(xyz / voxel) on the caller's array as it is (float64 from Open3D in the reference: no float32 rounding)
    xyz_in = np.ascontiguousarray(xyz, dtype=np.float64 if np.asarray(xyz).dtype == np.float64 else np.float32)
    coords, sel, counts, _ = voxelize([xyz_in], voxel_size, device)
    feats = torch.ones(coords.shape[0], 1, device=device)
    out = model(SparseTensor(feats, coords=coords, batch_size=1).to(device))
    return xyz[sel.cpu().numpy()], out.F


def transform_point_cloud(x1, R, t, data_type="numpy"):
    """scripts/utils.py:125-145: (R x1^T + t)^T for one cloud x1 [n, 3]"""
    assert data_type in ["numpy", "torch"]
    if data_type == "numpy":
        return (np.matmul(R, x1.transpose()) + t).transpose()
    return (torch.matmul(R, x1.transpose(1, 0)) + t).transpose(1, 0)
