"""lib.utils — the reference's numerics/utility surface (lib/utils.py).

Hot-path functions run on MI355X through libmvreg_hip.so:
  kabsch_transformation_estimation  (utils.py:164-237)  -> mvr_procrustes[_f64]
Pair building / filtering-input helpers keep the reference's tensor contract
(utils.py:850-932); the fused pipeline in lib.pairwise never materialises
them.  Host-side helpers (config, trajectory I/O and the registration
metrics of utils.py:438-637) are plain Python/numpy re-implementations.
"""
import logging
import math
import os
import re
import time
from itertools import combinations

import numpy as np
import torch
import yaml

from lib import _native as N


# --------------------------------------------------------------------------- config / files
def load_config(path):
    """utils.py:19-33: YAML config -> dict (safe loader)."""
    with open(path, "r") as f:
        return yaml.safe_load(f)


def load_point_cloud(file, data_type="numpy"):
    """utils.py:36-55 (open3d read) -> our PLY reader; returns float64 [N,3] like o3d."""
    assert data_type in ["numpy"], "open3d point cloud objects are not available; use data_type='numpy'"
    from lib.ply import read_ply_xyz
    return read_ply_xyz(file).astype(np.float64)


def sorted_alphanum(file_list_ordered):
    def key(s):
        return [int(tok) if tok.isdigit() else tok for tok in re.split("([0-9]+)", s)]
    return sorted(file_list_ordered, key=key)


def get_file_list(path, extension=None):
    files = [os.path.join(path, f) for f in os.listdir(path) if os.path.isfile(os.path.join(path, f))]
    if extension is not None:
        files = [f for f in files if os.path.splitext(f)[1] == extension]
    return sorted_alphanum(files)


def get_folder_list(path):
    return sorted_alphanum([os.path.join(path, f) for f in os.listdir(path) if os.path.isdir(os.path.join(path, f))])


def ensure_dir(path):
    os.makedirs(path, mode=0o755, exist_ok=True)


# --------------------------------------------------------------------------- rigid-motion numerics
def rotation_error(R1, R2):
    """utils.py:122-145: angle of R1^T R2 in degrees, [b,1]."""
    Rr = torch.matmul(R1.transpose(1, 2), R2)
    tr = Rr.diagonal(dim1=1, dim2=2).sum(-1)
    e = torch.clamp((tr - 1) / 2, -1, 1).unsqueeze(1)
    return torch.acos(e) * (180.0 / math.pi)


def translation_error(t1, t2):
    """utils.py:148-161."""
    return torch.norm(t1 - t2, dim=(1, 2))


def kabsch_transformation_estimation(x1, x2, weights=None, normalize_w=True, eps=1e-7, best_k=0, w_threshold=0):
    """Weighted Kabsch on MI355X (utils.py:164-237).  x1, x2 [b,n,3], weights [b,n].
    Returns (R [b,3,3], t [b,3,1], res [b,n], gradient_not_valid: bool)."""
    N.require_hip(x1)
    dt = x1.dtype
    if dt not in (torch.float32, torch.float64):
        raise TypeError("kabsch_transformation_estimation: float32/float64 only")
    B, Np, _ = x1.shape
    x1c = x1.contiguous()
    x2c = x2.to(dt).contiguous()
    w = None
    if weights is not None:
        w = weights.to(dt).contiguous().clone()
    normalize = bool(normalize_w)
    if best_k > 0 or w_threshold > 0:
        # rarely used reference options (no caller passes them): applied as in
        # utils.py:187-200 on the host side of the call, then an un-normalised solve
        if w is None:
            w = torch.ones(B, Np, dtype=dt, device=x1.device)
        if normalize:
            w = w / (w.sum(dim=1, keepdim=True) + eps)
            normalize = False
        if best_k > 0:
            idx = torch.topk(w[0], best_k).indices   # the reference selects on batch 0 only
            w, x1c, x2c = w[:, idx].contiguous(), x1c[:, idx].contiguous(), x2c[:, idx].contiguous()
            Np = best_k
        if w_threshold > 0:
            w = torch.where(w < w_threshold, torch.zeros_like(w), w)
    R = torch.empty(B, 3, 3, dtype=dt, device=x1.device)
    t = torch.empty(B, 3, 1, dtype=dt, device=x1.device)
    res = torch.empty(B, Np, dtype=dt, device=x1.device)
    status = torch.zeros(B, dtype=torch.int32, device=x1.device)
    L = N.lib()
    fn = L.mvr_procrustes if dt == torch.float32 else L.mvr_procrustes_f64
    N.check(fn(N.ptr(x1c), N.ptr(x2c), Np * 3, 3, N.ptr(w), Np, None, None, 0, B, Np, int(normalize), eps,
               N.ptr(R), N.ptr(t), N.ptr(res), Np, None, 0, N.ptr(status), 0, N.stream()), "mvr_procrustes")
    return R, t, res, bool(status.any().item())


def transformation_residuals(x1, x2, R, t):
    """utils.py:240-256: ||R x1 + t - x2|| per point."""
    x2r = torch.matmul(R, x1.transpose(1, 2)) + t
    return torch.norm(x2r.transpose(1, 2) - x2, dim=2)


def transform_point_cloud(x1, R, t):
    """utils.py:258-271."""
    return (torch.matmul(R, x1.transpose(1, 2)) + t).transpose(1, 2)


def _rows3(x):
    """(tensor, batch stride, row stride) of a [b, n, 3] float32 view whose 3 coordinates are contiguous."""
    if x.dim() != 3 or x.shape[2] != 3 or x.dtype != torch.float32:
        raise TypeError("expected a float32 [b, n, 3] tensor, got %s %s" % (x.dtype, tuple(x.shape)))
    if x.stride(2) != 1 or x.stride(1) < 3:
        x = x.contiguous()
    return x, x.stride(0), x.stride(1)


def knn_point(k, pos1, pos2):
    """utils.py:274-299: (squared distances, indices) [b, m, k] of the k nearest pos1 [b, n, 3] points for each pos2
    [b, m, 3] point, nearest first.  k = 1 (the reference's only use, extract_mutuals) is csrc/knn.hip mvr_knn1 in
    the reference's fp32 arithmetic without materialising the [b, m, n, 3] repeats; k > 1 evaluates the same
    expression in query chunks with torch.topk on the device.
    Device contract: pos1 on the HIP device (the op has no CPU path; CPU inputs raise), pos2 moved to it; results
    on that device.  NaN: a NaN distance is never selected by k = 1 (strict '<' scan; an all-NaN row returns
    index 0 and distance inf) where the reference's topk would return it; k > 1 keeps topk's NaN ordering."""
    N.require_hip(pos1)
    pos2 = pos2.to(pos1.device)
    B, n, _ = pos1.shape
    m = pos2.shape[1]
    if k == 1:
        p1, s1b, s1r = _rows3(pos1)
        p2, s2b, s2r = _rows3(pos2)
        d = torch.empty(B, m, 1, dtype=torch.float32, device=pos1.device)
        idx = torch.empty(B, m, 1, dtype=torch.int64, device=pos1.device)
        if B and m:
            N.check(N.lib().mvr_knn1(N.ptr(p1), s1b, s1r, N.ptr(p2), s2b, s2r, B, n, m, N.ptr(d), N.ptr(idx),
                                     N.stream()), "mvr_knn1")
        return d, idx
    vals, idxs = [], []
    step = max(1, (1 << 26) // max(1, B * n * 3))
    for q0 in range(0, m, step):
        q = pos2[:, q0:q0 + step]
        d = pos1[:, None, :, :] - q[:, :, None, :]
        dist = -((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2])   # the reference's order
        v, i = dist.topk(k=k, dim=-1)
        vals.append(-v)
        idxs.append(i)
    return torch.cat(vals, 1), torch.cat(idxs, 1)


def extract_mutuals(x1, x2, x1_soft_matches, x2_soft_matches, threshold=0.05):
    """utils.py:822-848: mutuals [b, n] float32, 1 where x1[i]'s soft match, snapped to its nearest x2 point j, maps
    back (x2_soft_matches[j]) to within `threshold` of x1[i].  One csrc/knn.hip mvr_mutuals launch (NN search,
    gather and threshold fused).  The reference fills a host tensor from a device mask (which fails for CUDA
    inputs); the flags stay on the inputs' device here (x1 on the HIP device; CPU inputs raise — INTEGRATION.md)."""
    N.require_hip(x1)
    B, Np, _ = x1.shape
    dev = x1.device
    a, ab, ar = _rows3(x1)
    b, bb, br = _rows3(x2.to(dev))
    c, cb, cr = _rows3(x1_soft_matches.to(dev))
    d, db, dr = _rows3(x2_soft_matches.to(dev))
    out = torch.empty(B, Np, dtype=torch.float32, device=dev)
    if B and Np:
        thr2 = float(np.float32(threshold ** 2))
        N.check(N.lib().mvr_mutuals(N.ptr(a), ab, ar, N.ptr(b), bb, br, N.ptr(c), cb, cr, N.ptr(d), db, dr, B, Np,
                                    thr2, N.ptr(out), None, N.stream()), "mvr_mutuals")
    return out


def pair_index(B, device=None):
    """All C(B,2) fragment pairs in lexicographic order (utils.py:873-876), int64 [P,2]."""
    pairs = torch.tensor(list(combinations(range(B), 2)), dtype=torch.long).reshape(-1, 2)
    if device is not None and torch.device(device).type == "cuda":
        # pinned + non_blocking: a pageable upload would block the host until the stream's queued work is done
        return pairs.pin_memory().to(device, non_blocking=True)
    return pairs.to(device) if device is not None else pairs


def extract_overlaping_pairs(xyz, feat, conectivity_info=None):
    """utils.py:850-885 (reference contract: materialises [P,n,*] tensors)."""
    if conectivity_info is None or (not torch.is_tensor(conectivity_info) and not conectivity_info):
        conectivity_info = pair_index(xyz.shape[0], xyz.device)
    ci = conectivity_info.to(xyz.device).long()
    return (torch.index_select(xyz, 0, ci[:, 0]), torch.index_select(xyz, 0, ci[:, 1]),
            torch.index_select(feat, 0, ci[:, 0]), torch.index_select(feat, 0, ci[:, 1]))


def extract_transformation_matrices(T0, indices):
    """utils.py:935-965: relative poses T_i T_j^-1 for the listed pairs (host)."""
    ind = indices.detach().cpu().numpy()
    T = T0.detach().cpu().numpy()
    rots, trans = [], []
    for i, j in ind:
        M = T[4 * i:4 * i + 4] @ np.linalg.inv(T[4 * j:4 * j + 4])
        rots.append(M[:3, :3])
        trans.append(M[:3, 3])
    return torch.from_numpy(np.asarray(rots)).to(T0), torch.from_numpy(np.asarray(trans)).unsqueeze(-1).to(T0)


def construct_filtering_input_data(xyz_s, xyz_t, data, overlapped_pair_tensors, dist_th=0.05, mutuals_flag=None):
    """utils.py:888-932 — the OANet input dict {xs [b,1,n,6|7], ys, ts, Rs}."""
    if "T_global_0" in data:
        Rs, ts = extract_transformation_matrices(data["T_global_0"], overlapped_pair_tensors)
        ys = transformation_residuals(xyz_s, xyz_t, Rs, ts)
    else:
        ys = torch.zeros(xyz_s.shape[0], xyz_s.shape[1], 1)
        Rs = torch.eye(3).unsqueeze(0).repeat(xyz_s.shape[0], 1, 1)
        ts = torch.zeros(xyz_s.shape[0], 3, 1)
    xs = torch.cat((xyz_s, xyz_t), dim=-1)
    if mutuals_flag is not None:
        xs = torch.cat((xs, mutuals_flag.reshape(xs.shape[0], xs.shape[1], 1).to(xs)), dim=-1)
    return {"xs": xs.unsqueeze(1), "ys": ys, "ts": ts, "Rs": Rs}


def pairwise_distance(src, dst, normalized_feature=False):
    """utils.py:968-992 (reference contract; the fused feature-NN kernel never materialises it)."""
    d = -torch.matmul(src, dst.permute(0, 2, 1))
    if not normalized_feature:
        d = 2 * d
        d += torch.sum(src ** 2, dim=-1)[:, :, None]
        d += torch.sum(dst ** 2, dim=-1)[:, None, :]
    return d


# --------------------------------------------------------------------------- 3DMatch / Redwood evaluation (host)
def read_trajectory(filename, dim=4):
    """utils.py:438-476: Redwood .log -> (keys [n,3] str, traj [n,dim,dim] float64)."""
    with open(filename) as f:
        lines = [ln for ln in f.read().splitlines() if ln.strip()]
    keys, mats = [], []
    for b in range(0, len(lines), dim + 1):
        keys.append([tok.strip() for tok in lines[b].split()[0:3]])
        mats.append([[float(v) for v in lines[b + 1 + r].split()[0:dim]] for r in range(dim)])
    return np.asarray(keys), np.asarray(mats, dtype=np.float64).reshape(-1, dim, dim)


def write_trajectory(traj, metadata, filename, dim=4):
    """utils.py:480-499.  The reference only writes rows whose overlap flag equals the
    STRING 'True' while its benchmark stores a bool (benchmark:220,224), so it writes an
    empty file; here both 'True' and True are accepted (documented deviation)."""
    with open(filename, "w") as f:
        for i in range(traj.shape[0]):
            flag = metadata[i][2]
            if flag is True or str(flag) == "True":
                f.write("\t".join(str(x) for x in metadata[i]) + "\n")
                f.write("\n".join("\t".join("{0:.12f}".format(v) for v in row) for row in traj[i].tolist()))
                f.write("\n")


def read_trajectory_info(filename, dim=6):
    """utils.py:502-532: Redwood .info -> (n_frames, cov [n,6,6])."""
    with open(filename) as f:
        lines = f.read().splitlines()
    n_pairs = len(lines) // 7
    assert len(lines) == 7 * n_pairs
    infos, n_frame = [], 0
    for i in range(n_pairs):
        _, _, n_frame = [int(v) for v in lines[7 * i].split()]
        infos.append([[float(v) for v in lines[7 * i + 1 + r].split()] for r in range(6)])
    return n_frame, np.asarray(infos, dtype=np.float64).reshape(-1, dim, dim)


def extract_corresponding_trajectors(est_pairs, gt_pairs, est_traj, gt_traj):
    """utils.py:534-560."""
    e = est_pairs[:, 0:2]
    ext_est, ext_gt = [], []
    for gi, pair in enumerate(gt_pairs[:, 0:2]):
        hit = np.where((e == pair).all(axis=1))[0]
        if hit.size:
            ext_gt.append(gt_traj[gi])
            ext_est.append(est_traj[hit[0]])
    return np.stack(ext_est, 0), np.stack(ext_gt, 0)


def mat2quat(M):
    """Rotation matrix -> quaternion (w, x, y, z) with w >= 0 (nibabel.quaternions.mat2quat
    convention: eigenvector of the symmetric K matrix, Bar-Itzhack)."""
    Qxx, Qyx, Qzx, Qxy, Qyy, Qzy, Qxz, Qyz, Qzz = np.asarray(M, dtype=np.float64).flat
    K = np.array([[Qxx - Qyy - Qzz, 0, 0, 0],
                  [Qyx + Qxy, Qyy - Qxx - Qzz, 0, 0],
                  [Qzx + Qxz, Qzy + Qyz, Qzz - Qxx - Qyy, 0],
                  [Qyz - Qzy, Qzx - Qxz, Qxy - Qyx, Qxx + Qyy + Qzz]]) / 3.0
    vals, vecs = np.linalg.eigh(K)
    q = vecs[[3, 0, 1, 2], np.argmax(vals)]
    if q[0] < 0:
        q = -q
    return q


def computeTransformationErr(trans, info):
    """utils.py:562-581: RMSE proxy e^T I e / I[0,0] with e = [t, q_xyz]."""
    t = trans[:3, 3]
    q = mat2quat(trans[:3, :3])
    er = np.concatenate([t, q[1:]], axis=0)
    return float((er.reshape(1, 6) @ info @ er.reshape(6, 1))[0, 0] / info[0, 0])


def evaluate_registration(num_fragment, result, result_pairs, gt_pairs, gt, gt_info, err2=0.2):
    """utils.py:584-637 (3DMatch/Redwood protocol; keeps the reference's quirk that GT
    pair index 0 is masked out because the mask stores the GT row index)."""
    err2 = err2 ** 2
    gt_mask = np.zeros((num_fragment, num_fragment), dtype=np.int64)
    for idx in range(gt_pairs.shape[0]):
        i, j = int(gt_pairs[idx, 0]), int(gt_pairs[idx, 1])
        if j - i > 1:
            gt_mask[i, j] = idx
    n_gt = np.sum(gt_mask > 0)
    good, n_res = 0, 0
    for idx in range(result_pairs.shape[0]):
        i, j = int(result_pairs[idx, 0]), int(result_pairs[idx, 1])
        if j - i > 1:
            n_res += 1
            gi = gt_mask[i, j]
            if gi > 0:
                p = computeTransformationErr(np.linalg.inv(gt[gi]) @ result[idx], gt_info[gi])
                if p <= err2:
                    good += 1
    if n_res == 0:
        n_res += 1e6
    return good * 1.0 / n_res, good * 1.0 / n_gt


RANSAC_N, RANSAC_DIST, RANSAC_ITERS = 4, 0.05, 2500   # utils.py:688,701-705: min(50000, 2500) iterations


def run_ransac_batch(xyz_i, xyz_j, counts=None, seed=0, ransac_n=RANSAC_N, max_dist=RANSAC_DIST,
                     iters=RANSAC_ITERS, device=None, return_all=False):
    """Batched RANSAC over correspondences (csrc/procrustes.hip mvr_ransac): xyz_i, xyz_j [P, n, 3]
    (torch or numpy; computed in fp64 as Open3D's Vector3d), counts [P] valid rows per pair (default n).
    Returns T [P, 4, 4] float64 numpy (x_j ~ T x_i), and with return_all also fitness, rmse, best_iter."""
    from lib import _native as N
    N.require_hip()
    dev = device or torch.device("cuda", torch.cuda.current_device())
    x1 = torch.as_tensor(xyz_i).to(dev, torch.float64).contiguous()
    x2 = torch.as_tensor(xyz_j).to(dev, torch.float64).contiguous()
    if x1.dim() != 3 or x1.shape != x2.shape or x1.shape[-1] != 3:
        raise ValueError("xyz_i / xyz_j must both be [P, n, 3]")
    P, n = x1.shape[0], x1.shape[1]
    cnt = torch.full((P,), n, dtype=torch.int32) if counts is None else torch.as_tensor(counts).to(torch.int32)
    if cnt.numel() != P or bool((cnt < 0).any()) or bool((cnt > n).any()):
        raise ValueError("counts must be [P] with 0 <= counts <= n")
    cnt = cnt.to(dev)
    T = torch.empty(P, 4, 4, dtype=torch.float64, device=dev)
    fit = torch.empty(P, dtype=torch.float64, device=dev)
    rmse = torch.empty(P, dtype=torch.float64, device=dev)
    best = torch.empty(P, dtype=torch.int32, device=dev)
    L = N.lib()
    ws = N.workspace(L.mvr_ransac_workspace_bytes(P, iters), dev)
    N.check(L.mvr_ransac(N.ptr(x1), N.ptr(x2), n * 3, N.ptr(cnt), P, ransac_n, iters, float(max_dist),
                         int(seed) & 0xFFFFFFFFFFFFFFFF, N.ptr(T), N.ptr(fit), N.ptr(rmse), N.ptr(best), None,
                         N.ptr(ws), ws.numel(), N.stream()), "mvr_ransac")
    if return_all:
        return T.cpu().numpy(), fit.cpu().numpy(), rmse.cpu().numpy(), best.cpu().numpy()
    return T.cpu().numpy()


def run_ransac(xyz_i, xyz_j, seed=0):
    """utils.py:671-709: RANSAC-based estimate of the transformation mapping xyz_i [n,3] onto xyz_j [n,3]
    (correspondences are row-aligned), returned as a 4x4 float64 array.  Open3D seeds its draws from the
    clock; here the draws come from a counter-based stream keyed by `seed` (default 0: the same pair gives the
    same estimate whatever ran before it in the process)."""
    x1 = np.asarray(xyz_i, dtype=np.float64).reshape(1, -1, 3)
    x2 = np.asarray(xyz_j, dtype=np.float64).reshape(1, -1, 3)
    return run_ransac_batch(x1, x2, seed=seed)[0]


def compute_overlap_ratio(pc_i, pc_j, trans, method="3DMatch", voxel_size=0.025):
    """utils.py:713-786 overlap gate (host implementation: voxel downsample + KD-tree NN)."""
    from lib.overlap import overlap_ratio
    return overlap_ratio(pc_i, pc_j, trans, method, voxel_size)


class Timer(object):
    """utils.py:1019-1047 wall-clock timer (callers add device syncs where they need them)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.total_time, self.calls, self.start_time, self.diff, self.avg = 0.0, 0, 0.0, 0.0, 0.0

    def tic(self):
        self.start_time = time.time()

    def toc(self, average=True):
        self.diff = time.time() - self.start_time
        self.total_time += self.diff
        self.calls += 1
        self.avg = self.total_time / self.calls
        return self.avg if average else self.diff


logging.getLogger(__name__).addHandler(logging.NullHandler())
