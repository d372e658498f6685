"""Evaluation loaders (lib/data.py = reference lib/data.py:9-45, 164-227 + scripts/utils.py:146-197) on a
synthetic tree in the reference's layout: file order, metadata, mutual filtering, collation, scene_info,
skipping of finished scenes and the gt.log pair list."""
import os
import types

import numpy as np
import torch

from lib.data import PrecomputedPairwiseEvalDataset, collate_fn, make_pairwise_eval_data_loader
from lib.utils import write_trajectory


def _tree(root, n=50):
    rng = np.random.default_rng(0)
    for scene, nf in (("kitchen", 4), ("sun3d-hotel_uc-scan3", 3)):
        os.makedirs(os.path.join(root, "correspondences", scene))
        os.makedirs(os.path.join(root, "features", scene))
        os.makedirs(os.path.join(root, "raw_data", scene))
        for i in range(nf):
            np.savez(os.path.join(root, "features", scene, "%s_%03d.npz" % (scene, i)),
                     xyz=rng.normal(size=(100 + i, 3)).astype(np.float32))
        for i in range(nf):
            for j in range(i + 1, nf):
                np.savez(os.path.join(root, "correspondences", scene, "%s_%03d_%03d.npz" % (scene, i, j)),
                         x=rng.normal(size=(n, 6)).astype(np.float32),
                         mutuals=(rng.random((n, 1)) < 0.3).astype(np.float32))
        # gt.log with a subset of the pairs (Redwood format: "i j n" + 4 rows)
        with open(os.path.join(root, "raw_data", scene, "gt.log"), "w") as f:
            for i, j in ((0, 1), (1, 2)):
                f.write("%d\t%d\t%d\n" % (i, j, nf) + "\n".join(" ".join("1" if r == c else "0" for c in range(4))
                                                                  for r in range(4)) + "\n")


def _args(root, **kw):
    a = dict(source_path=root, mutuals=0, method="RegBlock", overwrite=False, only_gt_overlaping=False, batch_size=4)
    a.update(kw)
    return types.SimpleNamespace(**a)


def test_dataset_and_loader(tmp_path):
    root = str(tmp_path)
    _tree(root)
    ds = PrecomputedPairwiseEvalDataset(_args(root))
    assert len(ds) == 6 + 3
    s = ds[0]
    assert s["metadata"] == ["kitchen", "000", "001"] and s["xs"].shape == (1, 50, 6)
    assert s["xyz1"][0].shape == (100, 3) and s["xyz2"][0].shape == (101, 3) and int(s["idx"]) == 0
    assert ds[6]["metadata"] == ["sun3d-hotel_uc-scan3", "000", "001"]
    b = collate_fn([ds[i] for i in range(3)])
    assert b["xs"].shape == (3, 1, 50, 6) and b["xs"].dtype == torch.float32
    assert b["idx"].tolist() == [0, 1, 2] and len(b["xyz1"]) == 3 and b["metadata"][2] == ["kitchen", "000", "003"]
    loader, info = make_pairwise_eval_data_loader(_args(root), num_workers=0)
    assert info == {"kitchen": [0, 24], "sun3d-hotel_uc-scan3": [24, 36], "nr_examples": 9}
    assert [bb["xs"].shape[0] for bb in loader] == [4, 4, 1]


def test_mutuals_gt_pairs_and_finished_scenes(tmp_path):
    root = str(tmp_path)
    _tree(root)
    ds = PrecomputedPairwiseEvalDataset(_args(root, mutuals=1))
    with np.load(ds.files[0]) as d:
        m = d["mutuals"].astype(bool).reshape(-1)
        np.testing.assert_array_equal(ds[0]["xs"][0], d["x"][m])
    loader, _ = make_pairwise_eval_data_loader(_args(root, mutuals=1), num_workers=0)
    assert all(bb["xs"].shape[0] == 1 for bb in loader)
    ds = PrecomputedPairwiseEvalDataset(_args(root, only_gt_overlaping=True))
    assert [s["metadata"][1:] for s in (ds[i] for i in range(len(ds)))] == [["000", "001"], ["001", "002"]] * 2
    # a scene with results is skipped unless overwrite
    out = os.path.join(root, "results", "RegBlock", "all", "kitchen")
    os.makedirs(out)
    write_trajectory(np.eye(4)[None], [["0", "1", True]], os.path.join(out, "traj.txt"))
    assert len(PrecomputedPairwiseEvalDataset(_args(root))) == 3
    assert len(PrecomputedPairwiseEvalDataset(_args(root, overwrite=True))) == 9
    _, info = make_pairwise_eval_data_loader(_args(root), num_workers=0)
    assert info == {"sun3d-hotel_uc-scan3": [0, 12], "nr_examples": 3}
