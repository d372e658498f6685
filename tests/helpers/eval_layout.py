"""Synthetic evaluation data in the reference's on-disk layout (lib/data.py:164-223, scripts/extract_data.py):
correspondences/<scene>/<scene>_iii_jjj.npz (x [n, 6], mutuals [n, 1]), features/<scene>/<scene>_iii.npz (xyz),
raw_data/<scene>/gt.log (the true transformations) and gt.info (identity information matrices).  Every fragment
views the same point set (true overlap 1); correspondences are 40 % exact matches + uniform outliers."""
import os

import numpy as np

from synth import random_rotation


def write_log(path, pairs, mats, n):
    with open(path, "w") as f:
        for (i, j), T in zip(pairs, mats):
            f.write("%d\t%d\t%d\n" % (i, j, n))
            f.write("\n".join("\t".join("%.12f" % v for v in row) for row in T) + "\n")


def write_scene(root, scene="kitchen", n_frag=5, n_corr=800, seed=0, n_base=3000):
    rng = np.random.default_rng(seed)
    base = rng.uniform(-1.0, 1.0, (n_base, 3))
    poses = []
    for k in range(n_frag):
        P = np.eye(4)
        P[:3, :3], P[:3, 3] = random_rotation(rng), rng.normal(0, 0.5, 3)
        poses.append(P)
    frag = [(base - P[:3, 3]) @ P[:3, :3] for P in poses]          # inv(P) applied: fragment frame
    for d in ("correspondences", "features", "raw_data"):
        os.makedirs(os.path.join(root, d, scene))
    for k in range(n_frag):
        np.savez(os.path.join(root, "features", scene, "%s_%03d.npz" % (scene, k)), xyz=frag[k].astype(np.float32))
    pairs, gts = [], []
    for i in range(n_frag):
        for j in range(i + 1, n_frag):
            sel = rng.choice(n_base, n_corr, replace=False)
            x1, x2 = frag[i][sel].copy(), frag[j][sel].copy()
            out = rng.random(n_corr) > 0.4
            x2[out] = rng.uniform(-1.5, 1.5, (out.sum(), 3))
            np.savez(os.path.join(root, "correspondences", scene, "%s_%03d_%03d.npz" % (scene, i, j)),
                     x=np.concatenate([x1, x2], 1).astype(np.float32),
                     mutuals=(rng.random((n_corr, 1)) > 0.3).astype(np.float32))
            pairs.append((i, j))
            gts.append(np.linalg.inv(poses[i]) @ poses[j])                # fragment j -> fragment i
    write_log(os.path.join(root, "raw_data", scene, "gt.log"), pairs, gts, n_frag)
    with open(os.path.join(root, "raw_data", scene, "gt.info"), "w") as f:
        for i, j in pairs:
            f.write("%d\t%d\t%d\n" % (i, j, n_frag) + "\n".join(" ".join("1" if r == c else "0" for c in range(6))
                                                              for r in range(6)) + "\n")
    return pairs


# two scenes whose pairs (36 + 15 = 51) make loader batches of 32 straddle the scene boundary, as in the reference
TWO_SCENES = (("kitchen", 9, 0), ("sun3d-hotel_uc-scan3", 6, 1))


def write_eval(root, dataset="3d_match", scenes=TWO_SCENES, n_corr=600):
    for name, n_frag, seed in scenes:
        write_scene(os.path.join(root, dataset), scene=name, n_frag=n_frag, n_corr=n_corr, seed=seed)


def read_results(root, dataset, method, mutuals=False):
    """{scene: traj.txt bytes} of a run"""
    base = os.path.join(root, dataset, "results", method, "mutuals" if mutuals else "all")
    return {s: open(os.path.join(base, s, "traj.txt"), "rb").read() for s in sorted(os.listdir(base))}
