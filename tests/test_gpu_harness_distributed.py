"""The evaluation harness sharded over ranks with the REAL GPU work (north_star config 4: "full 3DMatch
eval, pair batch sharded across GPUs, all-gather of (R,t,conf)"): scripts/benchmark_pairwise_registration.main
under torchrun's environment, two ranks on the box's one GPU (gloo: RCCL refuses two ranks on one device, so the
all-gather is host-staged), each running OANet (the reference's eval/RegBlock.yaml, train-mode BatchNorm per loader
batch as the reference benchmark) + Procrustes + the GPU overlap gate on its block of whole 32-pair loader batches;
rank 0 writes traj.txt and the report.  The trajectories must be byte-identical to one process, and both ranks
return the same summary — over two scenes whose pairs make a batch straddle the scene boundary (51 pairs)."""
import json
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN

HERE = os.path.dirname(os.path.abspath(__file__))
HELPERS = os.path.join(HERE, "helpers")
if HELPERS not in sys.path:
    sys.path.insert(0, HELPERS)

pytestmark = pytest.mark.gpu

REGBLOCK = os.path.join(GOLDEN, "configs", "pairwise_registration", "eval", "RegBlock.yaml")


def _checkpoint(path):
    """random-init RegBlock weights (no download offline) in the reference's checkpoint layout {'model': ...}"""
    import torch
    import lib.config
    from lib.utils import load_config
    from synth import synth_state
    model = lib.config.get_model(load_config(REGBLOCK))
    st = synth_state({k: tuple(v.shape) for k, v in model.state_dict().items()}, seed=11)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    torch.save({"model": {k: torch.from_numpy(np.asarray(v)) for k, v in st.items()}}, path)


@pytest.mark.parametrize("method,extra", [("RegBlock", []), ("RegBlock", ["--refine"]),
                                          ("RANSAC", ["--mutuals"])])
def test_harness_two_ranks_equal_one_process(gpu, tmp_path, method, extra):
    from eval_layout import write_eval, read_results
    from test_harness_distributed import run_ranks
    ckpt = str(tmp_path / "ckpt" / "model.pt")
    _checkpoint(ckpt)
    one, many = str(tmp_path / "one"), str(tmp_path / "many")
    for root in (one, many):
        write_eval(root)

    def argv(root):
        a = ["--source_path", root, "--method", method, "--batch_size", "32", "--num_workers", "0",
             "--dist_backend", "gloo"] + extra
        return a + (["--model", ckpt] if method != "RANSAC" else [])
    s1 = run_ranks(1, one, GOLDEN, argv(one), stub=False, timeout=240)[0]
    s2 = run_ranks(2, many, GOLDEN, argv(many), stub=False, timeout=240)
    mut = "--mutuals" in extra
    r1, r2 = read_results(one, "3d_match", method, mut), read_results(many, "3d_match", method, mut)
    assert sorted(r1) == ["kitchen", "sun3d-hotel_uc-scan3"]
    assert r1 == r2                                                   # byte-identical trajectories
    dump = lambda s: json.dumps(s, sort_keys=True)                  # noqa: E731  (NaN medians compare as text)
    assert dump(s2[0]) == dump(s1) and dump(s2[1]) == dump(s1)
    if method == "RANSAC":
        assert s1["recall"] == 1.0, s1
