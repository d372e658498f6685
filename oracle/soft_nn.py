"""Feature-space (soft) nearest neighbour, sampler and pair builder restated in
numpy (TEST ORACLE ONLY).

soft_nn            <- /root/reference/lib/layers.py:44-88, lib/utils.py:968-992
sample_rand        <- lib/layers.py:108-154 (samp_type='rand', host numpy RNG)
pair_index         <- lib/utils.py:868-876 (itertools.combinations order)
filtering_input    <- lib/utils.py:888-932 (no GT branch)
"""
from itertools import combinations

import numpy as np


def pairwise_distance(src, dst):
    """lib/utils.py:968-992 (normalized_feature=False)."""
    d = -np.matmul(src, np.swapaxes(dst, 1, 2))
    d = 2 * d
    d = d + (src ** 2).sum(-1)[:, :, None]
    d = d + (dst ** 2).sum(-1)[:, None, :]
    return d


def soft_nn(x_f, y_f, y_c, corr_type="soft", st=False, temp=0.3, min_temp=1e-4):
    """lib/layers.py:44-88.  x_f [B,N,C], y_f [B,M,C], y_c [B,M,3] -> x_corr [B,N,3].
    soft: softmax(-d / max(temp^2, min_temp)); st: forward value is the one-hot argmax;
    hard: one-hot argmin(d)."""
    dt = x_f.dtype
    d = pairwise_distance(x_f, y_f)
    if corr_type == "soft":
        tau2 = max(np.float32(temp) ** 2, np.float32(min_temp))
        z = -d / dt.type(tau2)
        z = z - z.max(axis=2, keepdims=True)
        e = np.exp(z)
        y = e / e.sum(axis=2, keepdims=True)
        if st:
            idx = y.argmax(axis=2)
            return np.take_along_axis(y_c, idx[..., None], axis=1)
        return np.matmul(y, y_c)
    if corr_type == "hard":
        idx = d.argmin(axis=2)
        return np.take_along_axis(y_c, idx[..., None], axis=1)
    raise ValueError("soft_gumbel: use soft_nn_gumbel (its noise needs a seed and the fragment ids)")


def _mix32(x):
    """lowbias32 finalizer (csrc/feat_nn.hip nn_mix32), uint32 arithmetic"""
    x = np.asarray(x, dtype=np.uint32)
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint32(16))
        x = x * np.uint32(0x7feb352d)
        x = x ^ (x >> np.uint32(15))
        x = x * np.uint32(0x846ca68b)
        x = x ^ (x >> np.uint32(16))
    return x


def gumbel_noise(seed, src, tgt, Nq, Mt):
    """The counter-based Gumbel noise of mvr_feat_nn_gumbel (csrc/feat_nn.hip nn_gumbel_query / nn_gumbel_z) for the
    pair (query fragment src, target fragment tgt): g [Nq, Mt] = -ln(-ln u), u = ((hash >> 9) + 1/2) 2^-23 in
    float64.  The reference draws g from torch's RNG (F.gumbel_softmax, lib/layers.py:72-78); this restates the
    distribution, not the stream."""
    u32 = np.uint32
    lo, hi = u32(seed & 0xFFFFFFFF), u32((seed >> 32) & 0xFFFFFFFF)
    with np.errstate(over="ignore"):
        k = _mix32(lo ^ _mix32(hi + u32(0x9E3779B9) * u32(tgt & 0xFFFFFFFF)) ^ (u32(0x85EBCA77) * u32(src & 0xFFFFFFFF)))
        hq = _mix32(k ^ np.arange(Nq, dtype=np.uint32))
        x = _mix32(hq[:, None] + u32(0x9E3779B9) * np.arange(Mt, dtype=np.uint32)[None, :])
    u = ((x >> u32(9)).astype(np.float64) + 0.5) * 2.0 ** -23
    return -np.log(-np.log(u))


def soft_nn_gumbel(x_f, y_f, y_c, src, tgt, seed, st=False, temp=0.3, min_temp=1e-4):
    """lib/layers.py:72-78 with gumbel_noise: F.gumbel_softmax(-d, tau=max(temp^2, min_temp), hard=st) . y_c per
    batch row b (query fragment src[b], target fragment tgt[b]); st: the forward value of the straight-through
    one-hot (y_c at the noisy argmax).  float64."""
    d = pairwise_distance(x_f.astype(np.float64), y_f.astype(np.float64))
    tau = float(max(np.float32(temp) ** 2, np.float32(min_temp)))
    out = []
    for b in range(d.shape[0]):
        z = (-d[b] + gumbel_noise(seed, int(src[b]), int(tgt[b]), d.shape[1], d.shape[2])) / tau
        if st:
            out.append(y_c[b][z.argmax(axis=1)])
            continue
        z = z - z.max(axis=1, keepdims=True)
        e = np.exp(z)
        out.append((e / e.sum(axis=1, keepdims=True)) @ y_c[b].astype(np.float64))
    return np.stack(out)


def sample_rand(pts_list, targeted_num_points, rng=np.random):
    """lib/layers.py:128-148: per fragment, np.random.choice over its global row
    range, always drawing `targeted_num_points`, without replacement iff
    min(targeted, min(pts_list)) >= targeted.  Returns int64 [B, targeted]."""
    pts_list = [int(p) for p in pts_list]
    num_points = min(targeted_num_points, min(pts_list))
    out = []
    start = 0
    for n in pts_list:
        rng_range = np.arange(start, start + n)
        out.append(rng.choice(rng_range, targeted_num_points, replace=not (num_points >= targeted_num_points)))
        start += n
    return np.stack(out).astype(np.int64)


def pair_index(B):
    """lib/utils.py:873-876: all C(B,2) pairs in lexicographic order, [P,2] int64."""
    return np.asarray(list(combinations(range(B), 2)), dtype=np.int64).reshape(-1, 2)


def filtering_input(xyz_s, xyz_t):
    """lib/utils.py:888-932 without GT: xs [P,1,N,6], ys zeros [P,N,1], Rs I, ts 0."""
    P, N, _ = xyz_s.shape
    xs = np.concatenate([xyz_s, xyz_t], axis=-1)[:, None]
    return {"xs": xs, "ys": np.zeros((P, N, 1), np.float32),
            "Rs": np.tile(np.eye(3, dtype=np.float32), (P, 1, 1)), "ts": np.zeros((P, 3, 1), np.float32)}
