"""The reference's YAML configs, loaded unchanged (BASELINE north_star: "configs/pairwise_registration YAMLs ...
run unchanged").  tests/golden/configs/ holds the reference's configs/pairwise_registration/{demo/config.yaml,
eval/RegBlock.yaml} byte for byte; tests/golden/config_models.json records what the reference's own factory
(lib/utils.py:19-33 load_config -> lib/config.py:9-25 get_model -> lib/pairwise/config.py:7-37) builds from each
(tests/golden/make_golden.py --only configs).  CPU only: building the modules allocates parameters, no kernels."""
import json
import os

import pytest

from conftest import GOLDEN

CONFIGS = ("configs/pairwise_registration/demo/config.yaml", "configs/pairwise_registration/eval/RegBlock.yaml")


def _rec():
    with open(os.path.join(GOLDEN, "config_models.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("rel", CONFIGS)
def test_load_config_parses_reference_yaml(rel):
    from lib.utils import load_config
    cfg = load_config(os.path.join(GOLDEN, rel))
    assert cfg == _rec()[rel]["cfg"]


@pytest.mark.parametrize("rel", CONFIGS)
def test_get_model_from_reference_yaml(rel):
    """lib.config.get_model on the unchanged file builds the reference's PairwiseReg: same attributes, same
    filter attributes, and the reference filter's exact state-dict key -> shape map under 'filtering_module.'."""
    from lib.utils import load_config
    import lib.config as config
    rec = _rec()[rel]
    model = config.get_model(load_config(os.path.join(GOLDEN, rel)))
    want = rec["pairwise"]
    assert model.samp_type == want["samp_type"] and model.corr_type == want["corr_type"]
    assert model.precomputed_desc == want["precomputed_desc"]
    assert bool(model.mutuals) == want["mutuals"] and bool(model.train_descriptor) == want["train_descriptor"]
    if not want["precomputed_desc"]:
        assert model.sampler.targeted_num_points == want["targeted_num_points"]
        assert model.sampler.samp_type == want["sampler_samp_type"]
        assert model.feature_matching.corr_type == want["matching_corr_type"]
        assert bool(model.feature_matching.st) == want["matching_st"]
        assert type(model.descriptor_module).__name__ == "FCGFNet"
    else:
        assert model.descriptor_module is None
    f = model.filtering_module
    assert type(f).__name__ == rec["filter"]["class"]
    assert f.iter_num == rec["filter"]["iter_num"] and bool(f.side_channel) == rec["filter"]["side_channel"]
    fk = {k: list(v.shape) for k, v in f.state_dict().items()}
    assert fk == rec["filter"]["keys"]
    sd = model.state_dict()
    assert {k[len("filtering_module."):]: list(v.shape) for k, v in sd.items()
            if k.startswith("filtering_module.")} == rec["filter"]["keys"]


def test_harness_reads_method_yaml_from_cwd(monkeypatch):
    """benchmark:159 reads ./configs/pairwise_registration/eval/<method>.yaml relative to the working directory;
    the mirror does the same, and a missing file is an error (no built-in substitute configuration)."""
    import torch
    from scripts import benchmark_pairwise_registration as B
    monkeypatch.setattr(torch.nn.Module, "to", lambda self, *a, **k: self)
    monkeypatch.chdir(GOLDEN)
    m = B.load_model("RegBlock", None)
    assert {k[len("filtering_module."):]: list(v.shape) for k, v in m.state_dict().items()} == \
        _rec()[CONFIGS[1]]["filter"]["keys"]
    with pytest.raises(FileNotFoundError):
        B.load_model("OANet", None)
    m2 = B.load_model("Anything", None, cfg_path=os.path.join(GOLDEN, CONFIGS[1]))
    assert m2.precomputed_desc


def test_scripts_utils_host_helpers(tmp_path):
    """scripts/utils.py's host helpers (reference :16-41, :125-145)"""
    import numpy as np
    import torch
    from scripts.utils import read_txt, ensure_dir, transform_point_cloud
    d = tmp_path / "a" / "b"
    ensure_dir(str(d))
    ensure_dir(str(d))
    (d / "x.txt").write_text(" one \ntwo\n")
    assert read_txt(str(d / "x.txt")) == ["one", "two"]
    r = np.random.RandomState(0)
    x = r.rand(7, 3)
    R = np.linalg.qr(r.rand(3, 3))[0]
    t = r.rand(3, 1)
    np.testing.assert_allclose(transform_point_cloud(x, R, t), x @ R.T + t.T)
    xt = transform_point_cloud(torch.from_numpy(x), torch.from_numpy(R), torch.from_numpy(t), data_type="torch")
    np.testing.assert_allclose(xt.numpy(), x @ R.T + t.T)
