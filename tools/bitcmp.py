"""Bit-identity check between two builds of libmvreg_hip.so (tools' A/B variants, MVR_LIB).
  python tools/bitcmp.py dump <out.npz>      run the strict train-mode OANet fixture (32 pairs x 5000, both blocks:
                                             logits, scores, R, t) and one scene step of the bench workload (records
                                             of all 435 pairs), save them
  python tools/bitcmp.py cmp <a.npz> <b.npz> count the elements that differ bit for bit (exit 1 if any)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dump(path):
    import json
    import torch
    import bench
    from synth import synth_correspondences
    dev = torch.device("cuda", 0)
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "oanet_full_train_strict.npz")))
    p = json.loads(str(g["params"]))
    xs, _, _ = synth_correspondences(32, 5000, seed=p["xs_seed"], inlier_lo=p["inlier_lo"], inlier_hi=p["inlier_hi"])
    out, _ = bench._oanet_golden(dev, "oanet_full_train_strict.npz", p["weights_seed"], xs)
    res = {}
    for i in range(2):
        for k in ("logits", "scores", "rot_est", "trans_est"):
            res["%s%d" % (k, i)] = out[k][i].detach().cpu().numpy()
    wl = bench.SceneWorkload(dev, 0)
    with torch.no_grad():
        res["scene_records"] = wl.step().cpu().numpy()
    np.savez(path, **res)
    print("dumped", path, {k: v.shape for k, v in res.items()})


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        x, y = A[k], B[k]
        n = int((x.view(np.uint32) != y.view(np.uint32)).sum()) if x.dtype == np.float32 else int((x != y).sum())
        bad += n
        print("%-16s %8d of %9d differ, max |diff| %.3g" % (k, n, x.size, float(np.abs(x - y).max()) if x.size else 0.0))
    print("BIT-IDENTICAL" if bad == 0 else "DIFFERENT")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(1 if cmp(sys.argv[2], sys.argv[3]) else 0)
