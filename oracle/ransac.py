"""RANSAC over given correspondences restated in numpy (TEST ORACLE ONLY).

Follows /root/reference/lib/utils.py:671-709 (run_ransac), which calls Open3D 0.9.0.0
`registration_ransac_based_on_correspondence` (README.md:47 pins open3d 0.9.0.0; absent here, so its
arithmetic is restated from the published 0.9 source, not imported) with
TransformationEstimationPointToPoint(with_scaling=False), ransac_n = 4, max_correspondence_distance = 0.05 and
RANSACConvergenceCriteria(max_iteration=50000, max_validation=2500):

  * min(max_iteration, max_validation) = 2500 iterations; no correspondence checkers are given;
  * each iteration draws ransac_n correspondences WITH replacement (Open3D: std::rand() % n);
  * fit: Umeyama without scaling (Eigen::umeyama): sigma = sum_j (d_j - mu_d)(s_j - mu_s)^T / k = U S V^T,
    R = U diag(1, 1, sign(det U det V)) V^T, t = mu_d - R mu_s;
  * evaluation over ALL correspondences: inlier iff |R s_i + t - d_i|^2 < max_dist^2, fitness = inliers / n,
    inlier_rmse = sqrt(sum of inlier squared distances / inliers);
  * result = the first iteration that strictly improves (fitness, then rmse) on the running best, which
    starts at fitness 0 / rmse 0 / identity: the lexicographic best among hypotheses with an inlier, earliest
    on exact ties; identity when none or n < ransac_n.

Parity is "unpinned" against Open3D itself (clock-seeded draws, not importable here).  The draws are the
build's own counter stream (include/mvreg.h mvr_ransac), restated in `draws`; the evaluation repeats the
kernel's fp64 operation order (rounded ops, no fma) so counts and error sums are bit-comparable.
"""
import numpy as np

GOLDEN = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1


def splitmix64(z):
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9 & M64
    z = (z ^ (z >> 27)) * 0x94D049BB133111EB & M64
    return z ^ (z >> 31)


def draws(seed, p, it, k, n):
    """indices of draw j < k of iteration `it` of pair p (csrc/procrustes.hip ransac_draw)"""
    out = []
    for j in range(k):
        ctr = (p << 40) | (it << 8) | j
        out.append(splitmix64((seed + ctr * GOLDEN) & M64) % n)
    return out


def umeyama(src, dst):
    """Eigen::umeyama(src, dst, with_scaling=false) on k x 3 fp64 arrays: R [3,3], t [3]."""
    k = src.shape[0]
    ms = np.zeros(3)
    md = np.zeros(3)
    for j in range(k):            # sequential sums, as the kernel
        ms = ms + src[j]
        md = md + dst[j]
    ms = ms / k
    md = md / k
    H = np.zeros((3, 3))
    for r in range(3):
        for c in range(3):
            acc = 0.0
            for j in range(k):
                acc = acc + (dst[j, r] - md[r]) * (src[j, c] - ms[c])
            H[r, c] = acc / k
    U, S, Vt = np.linalg.svd(H)
    sg = -1.0 if np.linalg.det(U) * np.linalg.det(Vt) < 0 else 1.0
    R = U @ np.diag([1.0, 1.0, sg]) @ Vt
    t = md - R @ ms
    return R, t


def evaluate(x1, x2, R, t, max_dist):
    """(inliers, sum of inlier squared distances) of one hypothesis, in the kernel's operation order:
    y_e = ((R_e0 s_0 + R_e1 s_1) + R_e2 s_2) + t_e, d2 = ((df_0^2 + df_1^2) + df_2^2), sequential over rows."""
    y = [((R[e, 0] * x1[:, 0] + R[e, 1] * x1[:, 1]) + R[e, 2] * x1[:, 2]) + t[e] for e in range(3)]
    df = [y[e] - x2[:, e] for e in range(3)]
    d2 = ((0.0 + df[0] * df[0]) + df[1] * df[1]) + df[2] * df[2]
    m = d2 < max_dist * max_dist
    good = int(m.sum())
    err = float(np.add.accumulate(d2[m])[-1]) if good else 0.0   # sequential sum in row order
    return good, err


def select(cnt, err, n):
    """index of the best hypothesis (-1: none), fitness, rmse"""
    best, bkey = -1, None
    for i in range(len(cnt)):
        if cnt[i] <= 0:
            continue
        key = (-cnt[i], np.sqrt(err[i] / cnt[i]))
        if bkey is None or key < bkey:
            best, bkey = i, key
    if best < 0:
        return -1, 0.0, 0.0
    return best, cnt[best] / n, float(np.sqrt(err[best] / cnt[best]))


def ransac(x1, x2, seed=0, ransac_n=4, max_dist=0.05, iters=2500, p=0, hyps=None):
    """One pair: returns (T [4,4], fitness, rmse, best_iter, hypotheses [iters, 12], counts, errors).
    `hyps` (e.g. the GPU's exported hypotheses) replaces the oracle's own Umeyama fits in the evaluation."""
    x1 = np.asarray(x1, np.float64)
    x2 = np.asarray(x2, np.float64)
    n = x1.shape[0]
    T = np.eye(4)
    if n < ransac_n:
        return T, 0.0, 0.0, -1, None, None, None
    own = np.zeros((iters, 12))
    cnt = np.zeros(iters, np.int64)
    err = np.zeros(iters)
    for it in range(iters):
        idx = draws(seed, p, it, ransac_n, n)
        R, t = umeyama(x1[idx], x2[idx])
        own[it, :9] = R.reshape(-1)
        own[it, 9:] = t
        if hyps is not None:
            R, t = hyps[it, :9].reshape(3, 3), hyps[it, 9:]
        cnt[it], err[it] = evaluate(x1, x2, R, t, max_dist)
    b, fit, rmse = select(cnt, err, n)
    if b >= 0:
        h = own[b] if hyps is None else hyps[b]
        T[:3, :3] = h[:9].reshape(3, 3)
        T[:3, 3] = h[9:]
    return T, fit, rmse, b, own, cnt, err
