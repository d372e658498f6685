"""End-to-end PairwiseReg (FCGF -> Sampler -> feature NN -> OANet -> Procrustes)
on the GPU vs the CPU oracle composition, stage by stage (each oracle stage is
fed the GPU's previous-stage output so tolerances do not compound)."""
import numpy as np
import pytest

from synth import synth_scene_fragments, synth_state

pytestmark = pytest.mark.gpu


def _cfg(npts, st=False):
    return {"method": {"task": "pairwise", "descriptor_module": "fcgf", "filter_module": "oanet"},
            "misc": {"net_depth": 12, "clusters": 500, "iter_num": 1, "net_channel": 128, "use_gpu": True,
                     "normalize_weights": True},
            "data": {"use_mutuals": 0, "max_num_points": npts},
            "train": {"samp_type": "rand", "corr_type": "soft", "st_grad_flag": st}}


def _cond(xs, w):
    """(s2 + s3) / s1 of the weighted Kabsch covariance per pair (R's sensitivity to
    weight perturbations scales with its inverse)."""
    w = w.astype(np.float64) / (w.sum(1, keepdims=True) + 1e-7)
    x1, x2 = xs[..., :3].astype(np.float64), xs[..., 3:6].astype(np.float64)
    m1 = (w[..., None] * x1).sum(1, keepdims=True)
    m2 = (w[..., None] * x2).sum(1, keepdims=True)
    H = np.einsum("pn,pni,pnj->pij", w, x1 - m1, x2 - m2)
    s = np.linalg.svd(H, compute_uv=False)
    return (s[:, 1] + s[:, 2]) / s[:, 0]


def test_pairwise_reg_end_to_end_vs_oracle(gpu):
    import torch
    import lib.config
    from lib.sparse import voxelize
    from oracle.fcgf import fcgf_forward
    from oracle.soft_nn import sample_rand, soft_nn, pair_index
    from oracle.oanet import oanet_forward

    frags, _ = synth_scene_fragments(3, seed=9, n_pts=60000)
    npts = 1000
    # st=True: the forward value is the hard (argmax) match, so x2 spans the target fragment and the
    # Kabsch problems are well conditioned even with random descriptor weights
    model = lib.config.get_model(_cfg(npts, st=True))
    shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    st = synth_state(shapes, seed=11)
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    model = model.to(gpu).eval()
    coords, sel, counts, xyz = voxelize([torch.from_numpy(f) for f in frags], 0.025, gpu)
    data = {"pcd0": xyz, "sinput0_C": coords, "sinput0_F": torch.ones(coords.shape[0], 1, device=gpu),
            "pts_list": torch.tensor(counts)}
    with torch.no_grad():
        np.random.seed(41)
        fin, F0, _, reg = model(data)
    F0 = F0.cpu().numpy()
    dst = {k[len("descriptor_module."):]: np.asarray(v) for k, v in st.items() if k.startswith("descriptor_module.")}
    fst = {k[len("filtering_module."):]: np.asarray(v) for k, v in st.items() if k.startswith("filtering_module.")}
    # stage 1: FCGF
    Fo, _ = fcgf_forward(dst, coords.cpu().numpy(), np.ones((coords.shape[0], 1), np.float32))
    assert np.abs(F0 - Fo).max() < 2e-4
    # stage 2: sampling + all-pairs soft NN (oracle on the GPU features)
    np.random.seed(41)
    idx = sample_rand(counts, npts)
    X = xyz.cpu().numpy()[idx]
    Fs = F0[idx]
    pi = pair_index(len(counts))
    xc = soft_nn(Fs[pi[:, 0]], Fs[pi[:, 1]], X[pi[:, 1]], "soft", st=True, temp=0.3)
    xs = fin["xs"][:, 0].cpu().numpy()
    np.testing.assert_array_equal(xs[..., :3], X[pi[:, 0]])
    assert np.mean(np.any(xs[..., 3:] != xc, axis=-1)) < 1e-3      # argmax: exact up to fp32 near-ties
    # stage 3: OANet + Kabsch on the GPU's xs
    o = oanet_forward(fst, xs)
    good = np.ones(len(xs), bool)
    for i in range(2):
        sc = reg["scores"][i].cpu().numpy()
        np.testing.assert_allclose(sc[good], o["scores"][i][good], atol=2e-3)
        near = np.abs(o["scores"][i] - 0.5) < 1e-4
        assert np.array_equal((sc > 0.5)[good][~near[good]], (o["scores"][i] > 0.5)[good][~near[good]])
        good &= _cond(xs, o["scores"][i]) > 0.3
        assert good.sum() >= 1, "no well-conditioned pair to compare"
        np.testing.assert_allclose(reg["rot_est"][i].cpu().numpy()[good], o["rot_est"][i][good], atol=1e-4)
        np.testing.assert_allclose(reg["trans_est"][i].cpu().numpy()[good], o["trans_est"][i][good], atol=1e-4)
