"""Weighted Kabsch / Procrustes restated in numpy (TEST ORACLE ONLY).

Follows /root/reference/lib/utils.py:164-237 (kabsch_transformation_estimation)
and :240-256 (transformation_residuals), op for op, in the input dtype.
"""
import numpy as np


def transformation_residuals(x1, x2, R, t):
    """lib/utils.py:240-256: ||R x1 + t - x2|| per point. x [B,N,3], R [B,3,3], t [B,3,1]."""
    x2r = np.matmul(R, np.swapaxes(x1, 1, 2)) + t
    return np.linalg.norm(np.swapaxes(x2r, 1, 2) - x2, axis=2)


def kabsch(x1, x2, weights=None, normalize_w=True, eps=1e-7, diag_embed=False):
    """lib/utils.py:164-237.  Returns (R [B,3,3], t [B,3,1], res [B,N], flag).

    diag_embed=True materialises the N x N diagonal weight matrix exactly as the
    reference does (utils.py:209-212); used only by the CPU baseline timing,
    the result is identical up to summation order."""
    dt = x1.dtype
    B, N, _ = x1.shape
    if weights is None:
        weights = np.ones((B, N), dtype=dt)
    weights = weights.astype(dt)
    if normalize_w:                                                   # :187-189
        sw = weights.sum(axis=1, keepdims=True) + dt.type(eps)
        weights = weights / sw
    w = weights[:, :, None]                                          # :191
    den = w.sum(axis=1)[:, None, :] + dt.type(eps)                   # :203-204
    x1m = np.matmul(np.swapaxes(w, 1, 2), x1) / den
    x2m = np.matmul(np.swapaxes(w, 1, 2), x2) / den
    x1c = x1 - x1m
    x2c = x2 - x2m
    if diag_embed:                                                   # :209-212
        W = np.zeros((B, N, N), dtype=dt)
        idx = np.arange(N)
        W[:, idx, idx] = weights
        cov = np.matmul(np.swapaxes(x1c, 1, 2), np.matmul(W, x2c))
    else:
        cov = np.matmul(np.swapaxes(x1c, 1, 2), w * x2c)
    try:                                                             # :214-223
        u, s, vh = np.linalg.svd(cov)
    except np.linalg.LinAlgError:
        R = np.tile(np.eye(3, dtype=dt), (B, 1, 1))
        t = np.zeros((B, 3, 1), dtype=dt)
        return R, t, transformation_residuals(x1, x2, R, t), True
    v = np.swapaxes(vh, 1, 2)                                        # torch.svd returns V
    det = np.linalg.det(np.matmul(np.swapaxes(v, 1, 2), np.swapaxes(u, 1, 2)))   # :225
    D = np.zeros((B, 3, 3), dtype=dt)
    D[:, 0, 0] = 1
    D[:, 1, 1] = 1
    D[:, 2, 2] = det                                                 # :227
    R = np.matmul(v, np.matmul(D, np.swapaxes(u, 1, 2))).astype(dt)  # :229
    t = (np.swapaxes(x2m, 1, 2) - np.matmul(R, np.swapaxes(x1m, 1, 2))).astype(dt)   # :232
    res = transformation_residuals(x1, x2, R, t).astype(dt)          # :235
    return R, t, res, False
