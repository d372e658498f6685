"""PairwiseReg (reference lib/pairwise/__init__.py:15-142) on the GPU against the reference's own outputs and
against the CPU oracle composition.

* test_pairwise_reg_fake_descriptor_golden — the a11 composition compute_descriptors -> filter_correspondences
  on the HIP path (Sampler draws, device gather, fused feature-NN over the C(B,2) pair list writing xs, OANet,
  Procrustes) with a fixed feature table standing in for FCGF, checked against pairwise_fake_desc.npz, which the
  reference itself produced (tests/golden/make_golden.py).
* test_pair_order_and_filtering_input_layout_golden — a5 / a8: the pair list's lexicographic order and the
  [x_s | x_corr] layout of the filtering input the fused matcher writes, against pairs.npz (the reference's
  extract_overlaping_pairs + construct_filtering_input_data).  With one-hot descriptors shared by every fragment,
  hard matching maps point i of the source onto point i of the target, so x_corr = xyz_t exactly.
* test_pairwise_reg_end_to_end_vs_oracle — FCGF -> Sampler -> soft NN -> OANet -> Kabsch on the GPU against
  the numpy oracle, stage by stage (each oracle stage is fed the GPU's previous-stage output, so tolerances do
  not compound).  FCGF itself is parity-unpinned (MinkowskiEngine is absent): its oracle is our restatement.
"""
import numpy as np
import pytest

from conftest import golden
from synth import synth_scene_fragments, synth_state

pytestmark = pytest.mark.gpu


def _small_filter(gpu, seed):
    import torch
    from test_gpu_oanet import _shapes
    from lib.filtering.oanet import OANet
    cfg = {"misc": {"net_depth": 12, "clusters": 16, "iter_num": 1, "net_channel": 32, "use_gpu": True,
                    "normalize_weights": True}, "data": {"use_mutuals": 0}}
    net = OANet(cfg)
    st = synth_state(_shapes("small"), seed=seed)
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    return net.to(gpu).eval()


class _FixedDescriptor:
    """Stands in for FCGFNet the way make_golden.py's FakeDesc does: row r of the sparse input gets table[r]."""

    def __new__(cls, table):
        import torch

        class FixedDescriptor(torch.nn.Module):
            def __init__(self, t):
                super().__init__()
                self.table = torch.nn.Parameter(t, requires_grad=False)

            def forward(self, st):
                class R:
                    pass
                r = R()
                r.F = self.table[: st.F.shape[0]]
                return r
        return FixedDescriptor(table)


def test_pairwise_reg_fake_descriptor_golden(gpu):
    import torch
    from lib.pairwise import PairwiseReg
    g = golden("pairwise_fake_desc.npz")
    pts = [int(p) for p in g["pts"]]
    tot = sum(pts)
    desc = _FixedDescriptor(torch.from_numpy(g["table"])).to(gpu)
    model = PairwiseReg(desc, _small_filter(gpu, seed=9), gpu, samp_type="rand", corr_type="soft",
                        tgt_num_points=1000, straight_through_gradient=False)
    data = {"pcd0": torch.from_numpy(g["pcd"]).to(gpu), "sinput0_C": torch.zeros(tot, 4, dtype=torch.int32),
            "sinput0_F": torch.ones(tot, 1), "pts_list": torch.tensor(pts)}
    with torch.no_grad():
        np.random.seed(41)
        fin, F0, F1, reg = model(data)
    xs = fin["xs"].cpu().numpy()
    assert xs.shape == g["xs"].shape == (3, 1, 1000, 6)
    np.testing.assert_array_equal(xs[..., :3], g["xs"][..., :3])          # sampled source points: exact
    np.testing.assert_allclose(xs[..., 3:], g["xs"][..., 3:], atol=2e-5)   # soft NN coordinates (golden bound)
    # the reference's placeholders (lib/utils.py:910-913), host-side like there
    assert fin["ys"].shape == (3, 1000, 1) and fin["Rs"].shape == (3, 3, 3) and fin["ts"].shape == (3, 3, 1)
    for i in range(2):
        sc, ref = reg["scores"][i].cpu().numpy(), g["scores%d" % i]
        np.testing.assert_allclose(reg["logits"][i].cpu().numpy(), g["logits%d" % i], atol=5e-4, rtol=1e-4)
        np.testing.assert_allclose(sc, ref, atol=5e-4)
        near = np.abs(ref - 0.5) < 1e-4
        assert np.array_equal((sc > 0.5)[~near], (ref > 0.5)[~near])
        np.testing.assert_allclose(reg["rot_est"][i].cpu().numpy(), g["R%d" % i], atol=1e-4)
        np.testing.assert_allclose(reg["trans_est"][i].cpu().numpy(), g["t%d" % i], atol=1e-4)
    assert bool(reg["gradient_flag"]) == bool(g["gradient_flag"])


def test_pair_order_and_filtering_input_layout_golden(gpu):
    import torch
    from lib.layers import Soft_NN
    from lib.utils import pair_index
    g = golden("pairs.npz")
    B, n = g["xyz"].shape[:2]
    pairs = pair_index(B, gpu)
    P = pairs.shape[0]
    assert P == g["xyz_s"].shape[0] == B * (B - 1) // 2
    pi = pairs.cpu().numpy()
    np.testing.assert_array_equal(g["xyz"][pi[:, 0]], g["xyz_s"])     # lexicographic combinations order
    np.testing.assert_array_equal(g["xyz"][pi[:, 1]], g["xyz_t"])
    np.testing.assert_array_equal(g["feat"][pi[:, 1]], g["f_t"])
    f = np.zeros((B, n, 32), np.float32)
    f[:, np.arange(n), np.arange(n)] = 1.0                              # point i <-> point i in every fragment
    xs = torch.full((P, n, 6), float("nan"), device=gpu)
    Soft_NN("hard", st=False).to(gpu).match_pairs(torch.from_numpy(f).to(gpu), torch.from_numpy(g["xyz"]).to(gpu),
                                                  pairs.contiguous(), xs, n * 6, 6)
    np.testing.assert_array_equal(xs.unsqueeze(1).cpu().numpy(), g["xs"])


def _cfg(npts, st=False):
    return {"method": {"task": "pairwise", "descriptor_module": "fcgf", "filter_module": "oanet"},
            "misc": {"net_depth": 12, "clusters": 500, "iter_num": 1, "net_channel": 128, "use_gpu": True,
                     "normalize_weights": True},
            "data": {"use_mutuals": 0, "max_num_points": npts},
            "train": {"samp_type": "rand", "corr_type": "soft", "st_grad_flag": st}}


def _cond(xs, w):
    """(s2 + s3) / s1 of the weighted Kabsch covariance per pair (R's sensitivity to weight perturbations scales
    with its inverse)."""
    w = w.astype(np.float64) / (w.sum(1, keepdims=True) + 1e-7)
    x1, x2 = xs[..., :3].astype(np.float64), xs[..., 3:6].astype(np.float64)
    m1 = (w[..., None] * x1).sum(1, keepdims=True)
    m2 = (w[..., None] * x2).sum(1, keepdims=True)
    H = np.einsum("pn,pni,pnj->pij", w, x1 - m1, x2 - m2)
    s = np.linalg.svd(H, compute_uv=False)
    return (s[:, 1] + s[:, 2]) / s[:, 0]


@pytest.mark.parametrize("st", [True, False])
def test_pairwise_reg_end_to_end_vs_oracle(gpu, st):
    import torch
    import lib.config
    from lib.sparse import voxelize
    from oracle.fcgf import fcgf_forward, voxelize as ovox
    from oracle.soft_nn import sample_rand, soft_nn, pair_index
    from oracle.oanet import oanet_forward

    frags, _ = synth_scene_fragments(3, seed=9, n_pts=60000)
    npts = 1000
    model = lib.config.get_model(_cfg(npts, st=st))
    shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    sd = synth_state(shapes, seed=11)
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    model = model.to(gpu).eval()
    coords, sel, counts, xyz = voxelize([torch.from_numpy(f) for f in frags], 0.025, gpu)
    # stage 0: voxelisation (ME sparse_quantize semantics as restated by the oracle): bit-exact
    oc, osel, ocnt = ovox(frags, 0.025)
    np.testing.assert_array_equal(coords.cpu().numpy(), oc)
    np.testing.assert_array_equal(sel.cpu().numpy(), osel)
    assert list(counts) == list(ocnt)
    data = {"pcd0": xyz, "sinput0_C": coords, "sinput0_F": torch.ones(coords.shape[0], 1, device=gpu),
            "pts_list": torch.tensor(counts)}
    with torch.no_grad():
        np.random.seed(41)
        fin, F0, _, reg = model(data)
    F0 = F0.cpu().numpy()
    dst = {k[len("descriptor_module."):]: np.asarray(v) for k, v in sd.items() if k.startswith("descriptor_module.")}
    fst = {k[len("filtering_module."):]: np.asarray(v) for k, v in sd.items() if k.startswith("filtering_module.")}
    # stage 1: FCGF (our restatement of ME's sparse conv: parity unpinned)
    Fo, _ = fcgf_forward(dst, coords.cpu().numpy(), np.ones((coords.shape[0], 1), np.float32))
    assert np.abs(F0 - Fo).max() < 2e-4
    # stage 2: sampling (the reference's numpy draws) + all-pairs NN (oracle on the GPU features)
    np.random.seed(41)
    idx = sample_rand(counts, npts)
    X = xyz.cpu().numpy()[idx]
    Fs = F0[idx]
    pi = pair_index(len(counts))
    xc = soft_nn(Fs[pi[:, 0]], Fs[pi[:, 1]], X[pi[:, 1]], "soft", st=st, temp=0.3)
    xs = fin["xs"][:, 0].cpu().numpy()
    np.testing.assert_array_equal(xs[..., :3], X[pi[:, 0]])
    if st:   # forward value = the hard (argmax) match: exact up to fp32 near-ties
        assert np.mean(np.any(xs[..., 3:] != xc, axis=-1)) < 1e-3
    else:
        np.testing.assert_allclose(xs[..., 3:], xc, atol=2e-5)
    # stage 3: OANet + Kabsch on the GPU's xs
    _compare_filter(reg, oanet_forward(fst, xs), xs)


def _compare_filter(reg, o, xs):
    """OANet scores / masks / R / t of the GPU against the oracle run on the GPU's own filtering input.  R and t are
    compared on the pairs whose weighted Kabsch covariance is well conditioned in every block so far (R's
    sensitivity to weight perturbations scales with the inverse of _cond); at least one such pair must remain in
    EVERY block, so the comparison can never pass vacuously."""
    good = np.ones(len(xs), bool)
    for i in range(2):
        sc = reg["scores"][i].cpu().numpy()
        np.testing.assert_allclose(sc[good], o["scores"][i][good], atol=2e-3)
        near = np.abs(o["scores"][i] - 0.5) < 1e-4
        assert np.array_equal((sc > 0.5)[good][~near[good]], (o["scores"][i] > 0.5)[good][~near[good]])
        good &= _cond(xs, o["scores"][i]) > 0.3
        assert good.any(), "block %d: no well-conditioned pair left to compare R / t on" % i
        np.testing.assert_allclose(reg["rot_est"][i].cpu().numpy()[good], o["rot_est"][i][good], atol=1e-4)
        np.testing.assert_allclose(reg["trans_est"][i].cpu().numpy()[good], o["trans_est"][i][good], atol=1e-4)


@pytest.mark.parametrize("st", [False, True])
def test_config2_full_size_pair_end_to_end_vs_oracle(gpu, st):
    """BASELINE configs[1] at full size: ONE 3DMatch-scale pair (two synthetic fragments of 250 k raw points ->
    20,590 / 21,280 voxels at 0.025 m), the reference's demo config (configs/pairwise_registration/demo/config.yaml,
    unchanged: FCGF, rand 5000 samples, soft NN, RegBlock-size OANet; st_grad_flag False as shipped, and True),
    model.eval() as scripts/pairwise_demo.py:109-110, compute_descriptors -> filter_correspondences as :147-154.
    Every stage against the oracle (FCGF on its C + OpenMP backend), each fed the GPU's previous-stage output:
    voxels exact, descriptors <= 2e-4, samples exact, soft / st matches, OANet scores and masks, R and t <= 1e-4.
    Fragments seed 4 and weights seed 12 were chosen (a CPU oracle scan) so the single pair is well conditioned in
    both blocks of both modes: the R / t comparison cannot be skipped."""
    import torch
    import lib.config
    from lib.utils import load_config
    from lib.sparse import voxelize
    from oracle.fcgf import fcgf_forward, voxelize as ovox
    from oracle.soft_nn import sample_rand, soft_nn, pair_index
    from oracle.oanet import oanet_forward
    from test_gpu_benchmark_harness import DEMO_CFG
    cfg = load_config(DEMO_CFG)
    cfg["train"]["st_grad_flag"] = st
    npts = cfg["data"]["max_num_points"]
    assert npts == 5000 and cfg["misc"]["voxel_size"] == 0.025
    frags, _ = synth_scene_fragments(2, seed=4)
    model = lib.config.get_model(cfg)
    sd = synth_state({k: tuple(v.shape) for k, v in model.state_dict().items()}, seed=12)
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    model = model.to(gpu).eval()
    coords, sel, counts, xyz = voxelize([torch.from_numpy(f) for f in frags], 0.025, gpu)
    oc, osel, ocnt = ovox(frags, 0.025)
    np.testing.assert_array_equal(coords.cpu().numpy(), oc)
    np.testing.assert_array_equal(sel.cpu().numpy(), osel)
    assert list(counts) == list(ocnt) == [20590, 21280]
    data = {"pcd0": xyz, "sinput0_C": coords, "sinput0_F": torch.ones(coords.shape[0], 1, device=gpu),
            "pts_list": torch.tensor(counts)}
    with torch.no_grad():
        np.random.seed(41)
        fin, F0, _ = model.compute_descriptors(data)
        reg = model.filter_correspondences(fin)
    F0 = F0.cpu().numpy()
    dst = {k[len("descriptor_module."):]: np.asarray(v) for k, v in sd.items() if k.startswith("descriptor_module.")}
    fst = {k[len("filtering_module."):]: np.asarray(v) for k, v in sd.items() if k.startswith("filtering_module.")}
    Fo, _ = fcgf_forward(dst, oc, np.ones((len(oc), 1), np.float32), backend="c")
    assert np.abs(F0 - Fo).max() < 2e-4
    np.random.seed(41)
    idx = sample_rand(list(ocnt), npts)
    X = xyz.cpu().numpy()[idx]
    Fs = F0[idx]
    pi = pair_index(2)
    xc = soft_nn(Fs[pi[:, 0]], Fs[pi[:, 1]], X[pi[:, 1]], "soft", st=st, temp=0.3)
    xs = fin["xs"][:, 0].cpu().numpy()
    assert xs.shape == (1, npts, 6)
    np.testing.assert_array_equal(xs[..., :3], X[pi[:, 0]])
    if st:
        assert np.mean(np.any(xs[..., 3:] != xc, axis=-1)) < 1e-3
    else:
        np.testing.assert_allclose(xs[..., 3:], xc, atol=2e-5)
    _compare_filter(reg, oanet_forward(fst, xs), xs)
