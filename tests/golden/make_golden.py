#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ by importing the REFERENCE
implementation (read-only at /root/reference) on CPU.

This script is the only thing in the repo that touches /root/reference, and it
runs only in the build container (never on the GPU box).  It writes DATA
(inputs + the reference's outputs) as small .npz / .json fixtures; no
reference source is copied.

Module stubs (the reference imports packages that are absent here; none of
them is on the arithmetic path of the functions we capture):
  * open3d, nibabel  -> empty modules (used only for I/O / eval metrics)
  * MinkowskiEngine  -> SparseTensor/MinkowskiNetwork shells (FCGF is NOT run)
  * np.float/np.int  -> builtins (removed in numpy>=1.24, used in lib/utils.py)
  * Soft_NN device   -> 'cpu' (lib/layers.py:21 hard-codes 'cuda')

Usage:  python tests/golden/make_golden.py [--ref /root/reference]
"""
import argparse
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from synth import synth_state, synth_correspondences, unit_features  # noqa: E402


def install_stubs():
    import torch
    for name in ("open3d", "nibabel", "nibabel.quaternions", "coloredlogs"):
        sys.modules.setdefault(name, types.ModuleType(name))
    me = types.ModuleType("MinkowskiEngine")
    me.__path__ = []

    class SparseTensor:
        def __init__(self, feats=None, coords=None, **kw):
            self.F = feats
            self.C = coords

        def to(self, dev):
            return self

    class MinkowskiNetwork(torch.nn.Module):
        def __init__(self, D):
            super().__init__()
            self.D = D

    me.SparseTensor = SparseTensor
    me.MinkowskiNetwork = MinkowskiNetwork
    mef = types.ModuleType("MinkowskiEngine.MinkowskiFunctional")
    me.MinkowskiFunctional = mef
    sys.modules["MinkowskiEngine"] = me
    sys.modules["MinkowskiEngine.MinkowskiFunctional"] = mef
    np.float = float  # noqa
    np.int = int  # noqa


def small_cfg(net_channel=32, clusters=16, use_mutuals=0):
    return {"misc": {"net_depth": 12, "clusters": clusters, "iter_num": 1, "net_channel": net_channel,
                     "use_gpu": False, "normalize_weights": True},
            "data": {"use_mutuals": use_mutuals, "max_num_points": 5000},
            "method": {"task": "pairwise", "descriptor_module": None, "filter_module": "oanet"},
            "train": {"samp_type": "rand", "corr_type": "soft", "st_grad_flag": False}}


def load_state(module, seed, overrides=None):
    import torch
    shapes = {k: tuple(v.shape) for k, v in module.state_dict().items()}
    st = synth_state(shapes, seed=seed, overrides=overrides)
    module.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    return shapes


def oanet_outputs(out):
    d = {}
    for i in range(len(out["logits"])):
        d["logits%d" % i] = out["logits"][i].numpy()
        d["scores%d" % i] = out["scores"][i].numpy()
        d["R%d" % i] = out["rot_est"][i].numpy()
        d["t%d" % i] = out["trans_est"][i].numpy()
    d["latent"] = out["latent features"].numpy()
    d["gradient_flag"] = np.asarray(bool(out["gradient_flag"]))
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--only", default=None, help="comma-separated fixture groups to (re)write: kabsch, oanet, "
                    "oanet_full_train, oanet_full_train_strict, softnn, sampler, pairs, pairwise, mutuals, evalharness, "
                    "configs (default: all)")
    args = ap.parse_args()
    only = set(args.only.split(",")) if args.only else None

    def want(tag):
        return only is None or tag in only
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.path.insert(0, args.ref)
    install_stubs()
    import torch
    torch.set_num_threads(8)
    import lib.utils as U
    import lib.layers as L
    from lib.filtering import oanet as O

    out = args.out
    meta = {"generator": "tests/golden/make_golden.py", "reference": "zgojcic/3D_multiview_reg @ /root/reference",
            "torch": torch.__version__, "numpy": np.__version__, "fixtures": {}}
    mpath = os.path.join(out, "GOLDEN_META.json")
    if only is not None and os.path.exists(mpath):
        with open(mpath) as f:
            meta["fixtures"] = json.load(f)["fixtures"]

    # ---------------------------------------------------------------- Kabsch
    # lib/utils.py:164-237 (+ transformation_residuals :240-256)
    if want("kabsch"):
        kabsch_fixture(U, out, meta)

    # ---------------------------------------------------------------- OANet
    # lib/filtering/oanet.py:18-265
    if want("oanet"):
        oanet_fixtures(O, out, meta)
    if want("oanet_full_train"):
        oanet_full_train_fixture(O, out, meta)
    if want("oanet_full_train_strict"):
        oanet_full_train_strict_fixture(O, out, meta)
    if want("softnn"):
        softnn_fixture(L, out, meta)
    if want("sampler"):
        sampler_fixture(L, out, meta)
    if want("pairs"):
        pairs_fixture(U, out, meta)
    if want("pairwise"):
        pairwise_fixture(L, O, out, meta)
    if want("mutuals"):
        mutuals_fixture(U, out, meta)
    if want("evalharness"):
        evalharness_fixture(U, out, meta)
    if want("configs"):
        configs_fixture(U, args.ref, out, meta)
    with open(mpath, "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote golden fixtures to", out)


def kabsch_fixture(U, out, meta):
    import torch
    xs, Rg, tg = synth_correspondences(4, 5000, seed=11)
    r = np.random.RandomState(12)
    w = r.rand(4, 5000).astype(np.float32)
    w[1] = 0.0                                    # all-zero weight row
    w[2, r.rand(5000) < 0.7] = 0.0                # sparse weights
    fx = {"x1": xs[..., :3], "x2": xs[..., 3:], "w": w}
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        R, t, res, flag = U.kabsch_transformation_estimation(
            torch.from_numpy(xs[..., :3]).to(dt), torch.from_numpy(xs[..., 3:]).to(dt), torch.from_numpy(w).to(dt))
        fx["R_" + tag] = R.numpy()
        fx["t_" + tag] = t.numpy()
        fx["res_" + tag] = res.numpy()
        fx["flag_" + tag] = np.asarray(bool(flag))
    # unweighted call (weights=None)
    R, t, res, flag = U.kabsch_transformation_estimation(torch.from_numpy(xs[..., :3]), torch.from_numpy(xs[..., 3:]))
    fx["R_none"], fx["t_none"], fx["res_none"] = R.numpy(), t.numpy(), res.numpy()
    np.savez_compressed(os.path.join(out, "kabsch.npz"), **fx)
    meta["fixtures"]["kabsch.npz"] = "lib/utils.py:164-256 kabsch_transformation_estimation, fp32+fp64, zero row"


def run_oanet(O, cfg, xs, seed, train=False, overrides=None):
    import torch
    torch.manual_seed(0)
    net = O.OANet(cfg)
    shapes = load_state(net, seed, overrides)
    net.train(train)
    with torch.no_grad():
        o = net({"xs": torch.from_numpy(xs).unsqueeze(1)})
    return shapes, oanet_outputs(o)


def oanet_full_train_fixture(O, out, meta):
    """The mode the reference benchmark runs (scripts/benchmark_pairwise_registration.py:159-197 never calls
    model.eval(): BatchNorm normalises with the statistics of each 32-pair loader batch), RegBlock.yaml's network
    at full size.  xs is regenerated from its seed by the test (synth_correspondences(32, 5000, seed=33)); its
    sha1 is stored to prove it."""
    import hashlib
    xs, _, _ = synth_correspondences(32, 5000, seed=33)
    _, o = run_oanet(O, small_cfg(net_channel=128, clusters=500), xs, seed=7, train=True)
    o.pop("latent")
    np.savez_compressed(os.path.join(out, "oanet_full_train.npz"), xs_sha1=np.asarray(hashlib.sha1(xs.tobytes()).hexdigest()),
                        **o)
    meta["fixtures"]["oanet_full_train.npz"] = ("lib/filtering/oanet.py:218-265 train-mode BatchNorm (the benchmark's "
                                                "mode), RegBlock network C=128,K=500, B=32 x N=5000, weights "
                                                "synth_state(seed 7), xs = synth_correspondences(32,5000,seed=33)")


STRICT_TRAIN = {"weights_seed": 19, "xs_seed": 40, "inlier_lo": 0.2, "inlier_hi": 0.5}


def oanet_full_train_strict_fixture(O, out, meta):
    """The benchmark's mode (train-mode BatchNorm over one 32-pair batch, RegBlock network at full size) on a
    WELL-CONDITIONED input, so north_star's R/t <= 1e-4 can be enforced on every pair of both blocks.  The
    chaotic fixture above (oanet_full_train.npz) has pairs where the reference's own fp32 result sits 2.6e-4 from
    exact arithmetic; here the weights seed and the (structured, 20-50 % inlier) correspondences were chosen
    from a seed scan so that the reference's fp32 output is within 1e-5 of the reference's own float64 forward
    (the same module, net.double()) on every pair — that fp64 output is stored beside it (R%d_f64, t%d_f64)."""
    import hashlib
    import torch
    p = STRICT_TRAIN
    xs, _, _ = synth_correspondences(32, 5000, seed=p["xs_seed"], inlier_lo=p["inlier_lo"], inlier_hi=p["inlier_hi"])
    cfg = small_cfg(net_channel=128, clusters=500)
    _, o = run_oanet(O, cfg, xs, seed=p["weights_seed"], train=True)
    o.pop("latent")
    torch.manual_seed(0)
    net = O.OANet(cfg)
    load_state(net, p["weights_seed"])
    net = net.double().train(True)
    with torch.no_grad():
        o64 = net({"xs": torch.from_numpy(xs).double().unsqueeze(1)})
    for i in range(2):
        o["R%d_f64" % i] = o64["rot_est"][i].numpy()
        o["t%d_f64" % i] = o64["trans_est"][i].numpy()
        gap = max(np.abs(o["R%d" % i] - o["R%d_f64" % i]).max(), np.abs(o["t%d" % i] - o["t%d_f64" % i]).max())
        assert gap < 1e-5, ("not well conditioned", i, gap)
    np.savez_compressed(os.path.join(out, "oanet_full_train_strict.npz"),
                        xs_sha1=np.asarray(hashlib.sha1(xs.tobytes()).hexdigest()),
                        params=np.asarray(json.dumps(p, sort_keys=True)), **o)
    meta["fixtures"]["oanet_full_train_strict.npz"] = (
        "lib/filtering/oanet.py:218-265 train-mode BatchNorm, RegBlock network C=128,K=500, B=32 x N=5000, weights "
        "synth_state(seed 19), xs = synth_correspondences(32,5000,seed=40,inliers 20-50%%); reference fp32 output and "
        "the reference module's own float64 output (R%d_f64/t%d_f64): well conditioned, fp32-fp64 gap < 1e-5")


def oanet_fixtures(O, out, meta):
    keys = {}
    cfg = small_cfg()
    xs_s, _, _ = synth_correspondences(3, 300, seed=21)
    shapes, o = run_oanet(O, cfg, xs_s, seed=5)
    keys["small"] = {k: list(v) for k, v in shapes.items()}
    np.savez_compressed(os.path.join(out, "oanet_small_eval.npz"), xs=xs_s, **o)
    _, o = run_oanet(O, cfg, xs_s, seed=5, train=True)
    np.savez_compressed(os.path.join(out, "oanet_small_train.npz"), xs=xs_s, **o)
    _, o = run_oanet(O, cfg, xs_s, seed=5, overrides={"reg_init.output.bias": [-50.0]})
    assert o["scores0"].min() > 0, "guard should have fired"
    np.savez_compressed(os.path.join(out, "oanet_small_guard.npz"), xs=xs_s, **o)
    # NOTE: the side channel (use_mutuals == 2 -> 7 input channels, oanet.py:205) crashes in the
    # reference: OANBlock slices x2 = xs[..., 3:] (oanet.py:180) which is 4 wide for 7-channel input,
    # and kabsch's bmm then fails.  No fixture can be produced for it (reference defects).
    cfgF = small_cfg(net_channel=128, clusters=500)
    xs_f, _, _ = synth_correspondences(2, 5000, seed=31)
    shapesF, o = run_oanet(O, cfgF, xs_f, seed=7)
    keys["full"] = {k: list(v) for k, v in shapesF.items()}
    o.pop("latent")   # 5 MB; not needed at full size
    np.savez_compressed(os.path.join(out, "oanet_full_eval.npz"), xs=xs_f, **o)
    meta["fixtures"]["oanet_*.npz"] = ("lib/filtering/oanet.py:218-265; weights = synth_state(seed) by key; "
                                       "small: C=32,K=16,N=300,B=3 (eval / train-mode BN / zero-row guard / side channel); "
                                       "full: C=128,K=500,N=5000,B=2 eval")
    with open(os.path.join(out, "oanet_keys.json"), "w") as f:
        json.dump(keys, f, indent=0, sort_keys=True)


def softnn_fixture(L, out, meta):
    # ---------------------------------------------------------------- Soft_NN
    # lib/layers.py:10-88 + lib/utils.py:968-992
    import torch
    fs = unit_features(2, 1024, 32, seed=41)
    ft = unit_features(2, 1024, 32, seed=42)
    yc = np.random.RandomState(43).uniform(-2, 2, (2, 1024, 3)).astype(np.float32)
    fx = {"fs": fs, "ft": ft, "yc": yc}
    for mode, st in (("soft", False), ("soft", True), ("hard", False)):
        nn = L.Soft_NN(corr_type=mode, st=st, device="cpu")
        with torch.no_grad():
            x = nn(torch.from_numpy(fs), torch.from_numpy(ft), torch.from_numpy(yc))
        fx["x_%s%s" % (mode, "_st" if st else "")] = x.numpy()
    # a temperature below the floor (min_temp 1e-4 clamps tau^2)
    nn = L.Soft_NN(corr_type="soft", st=False, temp=0.005, device="cpu")
    with torch.no_grad():
        fx["x_soft_cold"] = nn(torch.from_numpy(fs), torch.from_numpy(ft), torch.from_numpy(yc)).numpy()
    np.savez_compressed(os.path.join(out, "softnn.npz"), **fx)
    meta["fixtures"]["softnn.npz"] = "lib/layers.py:44-88 soft / soft+st / hard, tau=0.3 and tau=0.005 (clamped)"


def sampler_fixture(L, out, meta):
    import torch
    # ---------------------------------------------------------------- Sampler
    # lib/layers.py:108-154 (host numpy RNG)
    fx = {}
    for tag, pts in (("demo", [18977, 19082]), ("short", [3000, 4500, 6000])):
        np.random.seed(41)
        tot = int(sum(pts))
        C = torch.zeros(tot, 3)
        C[:, 0] = torch.arange(tot, dtype=torch.float32)
        F = torch.zeros(tot, 4)
        s = L.Sampler(samp_type="rand", targeted_num_points=5000)
        sc, sf = s(C, F, torch.tensor(pts))
        fx["idx_" + tag] = sc[..., 0].numpy().astype(np.int64)
        fx["pts_" + tag] = np.asarray(pts)
    np.savez_compressed(os.path.join(out, "sampler.npz"), **fx)
    meta["fixtures"]["sampler.npz"] = "lib/layers.py:108-154 rand sampling indices after np.random.seed(41)"


def pairs_fixture(U, out, meta):
    import torch
    # ------------------------------------------- pairs + filtering input
    # lib/utils.py:850-932
    xyz = torch.from_numpy(np.random.RandomState(51).rand(5, 7, 3).astype(np.float32))
    ft_ = torch.from_numpy(np.random.RandomState(52).rand(5, 7, 4).astype(np.float32))
    xs_, xt_, fs_, ft2_ = U.extract_overlaping_pairs(xyz, ft_, None)
    fd = U.construct_filtering_input_data(xs_, xt_, {}, None)
    np.savez_compressed(os.path.join(out, "pairs.npz"), xyz=xyz.numpy(), feat=ft_.numpy(), xyz_s=xs_.numpy(),
                        xyz_t=xt_.numpy(), f_s=fs_.numpy(), f_t=ft2_.numpy(), xs=fd["xs"].numpy(),
                        ys=fd["ys"].numpy(), Rs=fd["Rs"].numpy(), ts=fd["ts"].numpy())
    meta["fixtures"]["pairs.npz"] = "lib/utils.py:850-932 extract_overlaping_pairs + construct_filtering_input_data"


def pairwise_fixture(L, O, out, meta):
    import torch
    cfg = small_cfg()
    # --------------------------- PairwiseReg composition with a fake descriptor
    # lib/pairwise/__init__.py:62-142 (compute_descriptors -> filter_correspondences)
    import functools
    L.Soft_NN.__init__ = functools.partialmethod(L.Soft_NN.__init__, device="cpu")
    import lib.pairwise as PW

    class FakeDesc(torch.nn.Module):
        """Stands in for FCGFNet: returns a fixed unit-norm feature per input row."""
        def __init__(self, table):
            super().__init__()
            self.table = table

        def forward(self, st):
            class R:
                pass
            r_ = R()
            r_.F = self.table[: st.F.shape[0]]
            return r_

    pts = [1500, 1800, 1200]
    tot = sum(pts)
    table = torch.from_numpy(unit_features(1, tot, 32, seed=61)[0])
    pcd = torch.from_numpy(np.random.RandomState(62).uniform(-1, 1, (tot, 3)).astype(np.float32))
    filt = O.OANet(cfg)
    load_state(filt, seed=9)
    filt.eval()
    model = PW.PairwiseReg(FakeDesc(table), filt, torch.device("cpu"), samp_type="rand", corr_type="soft",
                           tgt_num_points=1000, straight_through_gradient=False)
    with torch.no_grad():
        np.random.seed(41)
        fin, F0, F1, reg = model({"pcd0": pcd, "sinput0_C": torch.zeros(tot, 4, dtype=torch.int32),
                                  "sinput0_F": torch.ones(tot, 1), "pts_list": torch.tensor(pts)})
    o = oanet_outputs(reg)
    np.savez_compressed(os.path.join(out, "pairwise_fake_desc.npz"), pcd=pcd.numpy(), table=table.numpy(),
                        pts=np.asarray(pts), xs=fin["xs"].numpy(), **o)
    meta["fixtures"]["pairwise_fake_desc.npz"] = ("lib/pairwise/__init__.py:62-142 with a fixed feature table in place "
                                                  "of FCGF; np.random.seed(41); 3 fragments -> 3 pairs; small OANet seed 9")


def mutuals_fixture(U, out, meta):
    """lib/utils.py:274-299 knn_point and :822-848 extract_mutuals.  Soft matches are target points plus noise
    (so the NN snap is well defined) and the back-matches land at distances straddling the 5 cm threshold."""
    import torch
    r = np.random.RandomState(71)
    B, n = 3, 700
    x1 = r.uniform(-1, 1, (B, n, 3)).astype(np.float32)
    x2 = r.uniform(-1, 1, (B, n, 3)).astype(np.float32)
    perm = np.stack([r.permutation(n) for _ in range(B)])
    x1m = (np.take_along_axis(x2, perm[..., None], 1) + r.normal(0, 0.004, (B, n, 3))).astype(np.float32)
    x2m = r.uniform(-1, 1, (B, n, 3)).astype(np.float32)
    back = x1 + r.normal(0, 1, (B, n, 3)) * r.choice([0.005, 0.02, 0.2], (B, n, 1))
    for b in range(B):
        x2m[b, perm[b]] = back[b]
    t = {k: torch.from_numpy(v) for k, v in (("x1", x1), ("x2", x2), ("x1m", x1m), ("x2m", x2m))}
    mut = U.extract_mutuals(t["x1"], t["x2"], t["x1m"], t["x2m"])
    d1, i1 = U.knn_point(1, t["x2"], t["x1m"])
    d3, i3 = U.knn_point(3, t["x2"], t["x1m"][:, :50])
    np.savez_compressed(os.path.join(out, "mutuals.npz"), x1=x1, x2=x2, x1m=x1m, x2m=x2m, mutuals=mut.numpy(),
                        knn1_d=d1.numpy(), knn1_i=i1.numpy(), knn3_d=d3.numpy(), knn3_i=i3.numpy())
    meta["fixtures"]["mutuals.npz"] = ("lib/utils.py:274-299 knn_point (k=1 over 700 points, k=3 for 50 queries) and "
                                       ":822-848 extract_mutuals (threshold 0.05), B=3, RandomState(71)")


def _mat2quat(M):
    """nibabel.quaternions.mat2quat (absent here; the stub gets this restatement — Bar-Itzhack's eigenvector of
    the symmetric K matrix, w >= 0).  Everything around it in the fixture is the reference's own code; the
    quaternion itself stays parity-unpinned."""
    Qxx, Qyx, Qzx, Qxy, Qyy, Qzy, Qxz, Qyz, Qzz = np.asarray(M, dtype=np.float64).flat
    K = np.array([[Qxx - Qyy - Qzz, 0, 0, 0], [Qyx + Qxy, Qyy - Qxx - Qzz, 0, 0],
                  [Qzx + Qxz, Qzy + Qyz, Qzz - Qxx - Qyy, 0],
                  [Qyz - Qzy, Qzx - Qxz, Qxy - Qyx, Qxx + Qyy + Qzz]]) / 3.0
    vals, vecs = np.linalg.eigh(K)
    q = vecs[[3, 0, 1, 2], np.argmax(vals)]
    return -q if q[0] < 0 else q


def evalharness_fixture(U, out, meta):
    """The 3DMatch / Redwood evaluation harness (lib/utils.py:438-637): trajectory write / read, info read,
    extract_corresponding_trajectors, computeTransformationErr and evaluate_registration (with its quirk that GT
    row 0 is never counted: gt_mask stores the row index and tests > 0).  Text files the reference writes are kept
    as fixture data; the .info text is synthetic input."""
    import tempfile
    sys.modules["nibabel.quaternions"].mat2quat = _mat2quat
    U.nq = sys.modules["nibabel.quaternions"]
    r = np.random.RandomState(81)
    nfrag = 9

    def rigid(scale):
        a = r.normal(size=3)
        a = a / np.linalg.norm(a) * r.uniform(0, scale)
        K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
        th = np.linalg.norm(a)
        R = np.eye(3) + (np.sin(th) / max(th, 1e-12)) * K + ((1 - np.cos(th)) / max(th, 1e-12) ** 2) * K @ K
        T = np.eye(4)
        T[:3, :3] = R
        T[:3, 3] = r.uniform(-2, 2, 3)
        return T
    # GT pairs: row 0 is a non-consecutive pair (the quirk), consecutive pairs mixed in
    gt_pairs = [(0, 2), (0, 1), (1, 4), (2, 3), (2, 7), (3, 8), (4, 6), (5, 8), (6, 7), (1, 8)]
    gt_T = np.stack([rigid(3.0) for _ in gt_pairs])
    A = r.normal(size=(len(gt_pairs), 6, 6))
    gt_info = np.einsum("pij,pkj->pik", A, A) + 6 * np.eye(6)
    info_txt = "".join("%d\t%d\t%d\n" % (i, j, nfrag) + "".join("\t".join("%.10f" % v for v in row) + "\n"
                                                                  for row in gt_info[k])
                       for k, (i, j) in enumerate(gt_pairs))
    # estimates: every GT pair (some accurate, some off) plus extra non-GT pairs, in a shuffled order
    est_pairs, est_T = [], []
    for k, (i, j) in enumerate(gt_pairs):
        d = rigid([0.001, 0.05, 0.5][k % 3])
        d[:3, 3] = r.normal(0, [0.001, 0.05, 0.4][k % 3], 3)
        est_pairs.append((i, j))
        est_T.append(gt_T[k] @ d)
    for (i, j) in [(0, 5), (3, 4), (2, 6), (1, 3)]:
        est_pairs.append((i, j))
        est_T.append(rigid(3.0))
    order = r.permutation(len(est_pairs))
    est_pairs = np.asarray(est_pairs)[order]
    est_T = np.stack(est_T)[order]
    flags = np.where(r.rand(len(est_pairs)) < 0.8, "True", "False")
    meta_arr = np.asarray([[str(i), str(j), f] for (i, j), f in zip(est_pairs, flags)])
    with tempfile.TemporaryDirectory() as td:
        tp = os.path.join(td, "traj.txt")
        U.write_trajectory(est_T, meta_arr, tp)
        with open(tp) as f:
            traj_txt = f.read()
        keys, traj_read = U.read_trajectory(tp)
        gp = os.path.join(td, "gt.log")
        U.write_trajectory(gt_T, np.asarray([[str(i), str(j), "True"] for i, j in gt_pairs]), gp)
        with open(gp) as f:
            gt_txt = f.read()
        ip = os.path.join(td, "gt.info")
        with open(ip, "w") as f:
            f.write(info_txt)
        n_frame, info_read = U.read_trajectory_info(ip)
        gt_keys, gt_read = U.read_trajectory(gp)
    # as the reference benchmark does (benchmark_pairwise_registration.py:289-313): the string keys of both files
    ext_est, ext_gt = U.extract_corresponding_trajectors(keys, gt_keys, traj_read, gt_read)
    errs = np.asarray([U.computeTransformationErr(np.linalg.inv(gt_T[k]) @ est_T[order.tolist().index(k)],
                                                  gt_info[k]) for k in range(len(gt_pairs))])
    res = {}
    for err2 in (0.2, 0.05):
        p, rc = U.evaluate_registration(n_frame, traj_read, keys, gt_keys, gt_read, info_read, err2=err2)
        res["precision_%g" % err2], res["recall_%g" % err2] = p, rc
    np.savez_compressed(os.path.join(out, "evalharness.npz"), nfrag=nfrag, gt_pairs=np.asarray(gt_pairs), gt_T=gt_T,
                        gt_info=gt_info, info_txt=np.asarray(info_txt), est_pairs=est_pairs, est_T=est_T,
                        flags=flags, traj_txt=np.asarray(traj_txt), gt_txt=np.asarray(gt_txt), keys=keys,
                        gt_keys=gt_keys, gt_read=gt_read,
                        traj_read=traj_read, n_frame=n_frame, info_read=info_read, ext_est=ext_est, ext_gt=ext_gt,
                        errs=errs, **{k: np.asarray(v) for k, v in res.items()})
    meta["fixtures"]["evalharness.npz"] = ("lib/utils.py:438-637 write/read_trajectory, read_trajectory_info, "
                                           "extract_corresponding_trajectors, computeTransformationErr (mat2quat "
                                           "restated: unpinned), evaluate_registration at err2 0.2 / 0.05")


CONFIGS = ("configs/pairwise_registration/demo/config.yaml", "configs/pairwise_registration/eval/RegBlock.yaml")


def configs_fixture(U, ref, out, meta):
    """The reference's own YAMLs (data files, copied byte for byte to tests/golden/configs/) and what the
    reference's factory builds from each: lib/utils.py:19-33 load_config -> lib/config.py:9-25 get_model ->
    lib/pairwise/config.py:7-37.  Recorded per file: the parsed dict, the PairwiseReg attributes, the filter's
    attributes and its state-dict key -> shape map.  The demo config names the FCGF descriptor, which needs
    MinkowskiEngine (absent): the reference's get_descriptor is given a parameter-free placeholder, so the
    descriptor's keys stay parity-unpinned and only the rest of the model is recorded."""
    import functools
    import shutil
    import torch
    import lib.layers as L
    L.Soft_NN.__init__ = functools.partialmethod(L.Soft_NN.__init__, device="cpu")
    import lib.config as RC
    import lib.pairwise.config as RPC
    real_get_descriptor = RPC.get_descriptor
    RPC.get_descriptor = lambda cfg, device: (torch.nn.Identity() if cfg["method"]["descriptor_module"]
                                              else real_get_descriptor(cfg, device))
    rec = {}
    for rel in CONFIGS:
        src = os.path.join(ref, rel)
        dst = os.path.join(out, rel)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        shutil.copyfile(src, dst)
        cfg = U.load_config(src)
        model = RC.get_model(cfg)
        f = model.filtering_module
        r = {"cfg": cfg,
             "pairwise": {"samp_type": model.samp_type, "corr_type": model.corr_type,
                          "precomputed_desc": bool(model.precomputed_desc), "mutuals": bool(model.mutuals),
                          "train_descriptor": bool(model.train_descriptor)},
             "filter": {"class": type(f).__name__, "iter_num": int(f.iter_num), "side_channel": bool(f.side_channel),
                        "keys": {k: list(v.shape) for k, v in f.state_dict().items()}}}
        if not model.precomputed_desc:
            r["pairwise"].update({"targeted_num_points": int(model.sampler.targeted_num_points),
                                  "sampler_samp_type": model.sampler.samp_type,
                                  "matching_corr_type": model.feature_matching.corr_type,
                                  "matching_st": bool(model.feature_matching.st),
                                  "descriptor": "placeholder (FCGF needs MinkowskiEngine: keys unpinned)"})
        rec[rel] = r
    RPC.get_descriptor = real_get_descriptor
    with open(os.path.join(out, "config_models.json"), "w") as fh:
        json.dump(rec, fh, indent=0, sort_keys=True)
    meta["fixtures"]["config_models.json"] = ("lib/utils.py:19-33 load_config + lib/config.py:9-25 get_model on the "
                                              "reference's demo/config.yaml and eval/RegBlock.yaml (copied under "
                                              "configs/): PairwiseReg / filter attributes and filter state-dict keys")


if __name__ == "__main__":
    main()
