"""Correspondence producer on the GPU (replaces scripts/extract_data.py:122-200
run_correspondence_extraction for one scene): per fragment pair (i < j, the reference's loop
order) sample n rows of each fragment's FCGF descriptors with the host RNG exactly as the
reference draws them, take the two nearest neighbours in feature space both ways
(mvr_feat_knn2 on the split-bf16 matrix cores, fp64 distances of the chosen rows), and emit
the reference's npz fields:
    x        [n, 6]  (pc_1 keypoint matched to each pc_2 sample | pc_2 sample)
    mutuals  [n, 1]  1 where NN_2(NN_1(r)) == r (indexed by the pc_2 sample r)
    ratios   [n]     d1 / d2 of the pc_1 samples' two neighbours (indexed by pc_1 sample — the
                     reference's indexing, kept as is)
All pairs of a scene go through one kernel launch per direction."""
import numpy as np
import torch

from lib import _native as N


def sample_indices(n_rows, n, rng):
    """extract_data.py:158-166: without replacement when enough rows, else with replacement."""
    return rng.choice(n_rows, n, replace=n_rows < n)


def extract_correspondences(features, keypoints, n_correspondences=5000, rng=None, pairs=None):
    """features: list of [m_b, 32] float arrays/tensors (FCGF descriptors of fragment b), keypoints:
    list of [m_b, 3]; pairs: optional list of (i, j) (default: all i < j in the reference order);
    rng: numpy RandomState / module (default np.random, the reference's global state).
    Returns a list of dicts {'pair': (i, j), 'x', 'mutuals', 'ratios'} in pair order."""
    N.require_hip()
    rng = np.random if rng is None else rng
    B = len(features)
    if pairs is None:
        pairs = [(i, j) for i in range(B) for j in range(i + 1, B)]
    n = int(n_correspondences)
    dev = torch.device("cuda", torch.cuda.current_device())
    feats = [torch.as_tensor(np.asarray(f) if not torch.is_tensor(f) else f).to(dev, torch.float32) for f in features]
    kps = [np.asarray(k.cpu() if torch.is_tensor(k) else k) for k in keypoints]
    P = len(pairs)
    inds = []
    for i, j in pairs:                      # host RNG in the reference's draw order
        a = sample_indices(feats[i].shape[0], n, rng)
        b = sample_indices(feats[j].shape[0], n, rng)
        inds.append((a, b))
    # sampled descriptor sets: fragment 2p = pc_1 samples, 2p + 1 = pc_2 samples of pair p
    F = torch.empty(2 * P, n, 32, device=dev)
    for p, (i, j) in enumerate(pairs):
        F[2 * p] = feats[i][torch.from_numpy(inds[p][0]).to(dev)]
        F[2 * p + 1] = feats[j][torch.from_numpy(inds[p][1]).to(dev)]
    L = N.lib()
    fwd = torch.from_numpy(np.stack([np.arange(P) * 2, np.arange(P) * 2 + 1], 1).astype(np.int64)).to(dev)
    bwd = fwd.flip(1).contiguous()
    idx12 = torch.empty(P, n, 2, dtype=torch.int32, device=dev)
    d12 = torch.empty(P, n, 2, dtype=torch.float64, device=dev)
    idx21 = torch.empty(P, n, 2, dtype=torch.int32, device=dev)
    N.check(L.mvr_feat_knn2(N.ptr(F), n * 32, N.ptr(F), n * 32, N.ptr(fwd), P, n, n, 32, N.ptr(idx12), N.ptr(d12),
                            N.stream()), "mvr_feat_knn2")
    N.check(L.mvr_feat_knn2(N.ptr(F), n * 32, N.ptr(F), n * 32, N.ptr(bwd), P, n, n, 32, N.ptr(idx21), None,
                            N.stream()), "mvr_feat_knn2")
    i12 = idx12.long()
    i21 = idx21.long()
    ar = torch.arange(n, device=dev)
    mutual = (torch.gather(i12[:, :, 0], 1, i21[:, :, 0]) == ar).to(torch.float64)          # [P, n]
    ratios = (d12[:, :, 0] / d12[:, :, 1])                                                   # [P, n]
    i21_0 = i21[:, :, 0].cpu().numpy()
    mutual, ratios = mutual.cpu().numpy(), ratios.cpu().numpy()
    out = []
    for p, (i, j) in enumerate(pairs):
        k1 = kps[i][inds[p][0]]
        k2 = kps[j][inds[p][1]]
        out.append({"pair": (i, j), "x": np.concatenate([k1[i21_0[p]], k2], axis=1),
                    "mutuals": mutual[p][:, None], "ratios": ratios[p]})
    return out
