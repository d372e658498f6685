"""Correspondence producer restated on the CPU (TEST ORACLE ONLY) — scripts/extract_data.py:122-200
run_correspondence_extraction for a list of fragments, with the reference's own sklearn calls
(NearestNeighbors(n_neighbors=1, metric='minkowski', p=2).kneighbors(n_neighbors=2)) and its
index conventions (mutuals per pc_2 sample, ratios per pc_1 sample)."""
import numpy as np


def extract_pair(f1_all, k1_all, f2_all, k2_all, n, rng):
    from sklearn.neighbors import NearestNeighbors
    i1 = rng.choice(f1_all.shape[0], n, replace=f1_all.shape[0] < n)
    i2 = rng.choice(f2_all.shape[0], n, replace=f2_all.shape[0] < n)
    f1, f2, k1, k2 = f1_all[i1], f2_all[i2], k1_all[i1], k2_all[i2]
    nn = NearestNeighbors(n_neighbors=1, metric="minkowski", p=2)
    nn.fit(f2)
    d12, idx12 = nn.kneighbors(X=f1, n_neighbors=2, return_distance=True)
    nn.fit(f1)
    d21, idx21 = nn.kneighbors(X=f2, n_neighbors=2, return_distance=True)
    ol = np.where((idx12[idx21[:, 0], 0] - np.arange(f1.shape[0])) == 0)[0]
    mutuals = np.zeros((n, 1))
    mutuals[ol] = 1
    ratios = d12[:, 0] / d12[:, 1]
    x = np.concatenate((k1[idx21[:, 0], :], k2), axis=1)
    return {"x": x, "mutuals": mutuals, "ratios": ratios, "idx12": idx12, "idx21": idx21}


def extract_correspondences(features, keypoints, n, rng):
    B = len(features)
    return [dict(pair=(i, j), **extract_pair(features[i], keypoints[i], features[j], keypoints[j], n, rng))
            for i in range(B) for j in range(i + 1, B)]
