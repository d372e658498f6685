"""Evaluation data of the precomputed-correspondence benchmark (BASELINE configs[3]/[4]).

Restates the host-side loaders the benchmark uses (scripts/benchmark_pairwise_registration.py:33 ->
scripts/utils.py:146-197 make_pairwise_eval_data_loader -> lib/data.py:164-227 PrecomputedPairwiseEvalDataset,
collated by lib/data.py:9-45 collate_fn).  Same directory layout, file names, sample dicts and scene
bookkeeping, so `batch['xs']` goes straight into `OANet.forward` / `PairwiseReg.filter_correspondences`
and the per-pair records feed `lib.overlap` and the trajectory writer.  The training datasets of
lib/data.py (:48-160, :235-360) are out of scope (training).

Layout under `source_path`:
  correspondences/<scene>/<scene>_<iii>_<jjj>.npz   x [n, 6] (x_i | x_j), mutuals [n, 1] (scripts/extract_data.py)
  features/<scene>/<scene>_<iii>.npz                xyz [m, 3]
  raw_data/<scene>/gt.log                           (only_gt_overlaping)
  results/<method>/{all|mutuals}/<scene>/traj.txt   (scenes with results are skipped unless overwrite)
"""
import logging
import os

import numpy as np
import torch
import torch.utils.data as data

from lib.utils import get_file_list, get_folder_list, read_trajectory


def collate_fn(batch):
    """lib/data.py:9-45: numpy arrays -> float32 tensors, stacked per key; lists stay lists."""
    def to_tensor(x):
        if isinstance(x, torch.Tensor):
            return x
        if isinstance(x, np.ndarray):
            return torch.from_numpy(x).float()
        raise ValueError(f"Can not convert to torch tensor, {x}")

    out = {key: [] for key in batch[0]}
    for sample in batch:
        for key in sample:
            out[key].append(sample[key] if isinstance(sample[key], list) else to_tensor(sample[key]))
    for key in out:
        if isinstance(out[key][0], torch.Tensor):
            out[key] = torch.stack(out[key])
    return out


def _results_dir(args):
    """lib/data.py:172-173"""
    return os.path.join(args.source_path, "results", args.method) + ("/mutuals/" if args.mutuals else "/all/")


def _scene_files(args):
    """(scene name, [correspondence files]) for every scene still to be evaluated (lib/data.py:178-193)"""
    out = []
    save_path = _results_dir(args)
    for folder in get_folder_list(os.path.join(args.source_path, "correspondences")):
        scene = folder.split("/")[-1]
        if os.path.exists(os.path.join(save_path, scene, "traj.txt")) and not args.overwrite:
            logging.info("Trajectory for scene %s already exists and will not be recomputed.", scene)
            continue
        if args.only_gt_overlaping:
            gt_pairs, _ = read_trajectory(os.path.join(args.source_path, "raw_data", scene, "gt.log"))
            files = [os.path.join(folder, scene + "_{}_{}.npz".format(str(i).zfill(3), str(j).zfill(3)))
                     for i, j, _ in gt_pairs]
        else:
            files = get_file_list(folder)
        out.append((scene, files))
    return out


class PrecomputedPairwiseEvalDataset(data.Dataset):
    """lib/data.py:164-227: one sample per correspondence file:
    {'xs': [1, n, 6], 'metadata': [scene, idx_1, idx_2], 'idx': array(idx), 'xyz1': [xyz], 'xyz2': [xyz]};
    with args.mutuals == 1 only the mutual rows of x are kept (so n varies: batch size 1)."""

    def __init__(self, args):
        self.root = args.source_path
        self.use_mutuals = args.mutuals
        logging.info("Loading the eval data from %s!", self.root)
        self.files = [f for _, files in _scene_files(args) for f in files]

    def __getitem__(self, idx):
        curr_file = self.files[idx]
        with np.load(curr_file, allow_pickle=False) as d:
            xs = d["x"]
            mutuals = d["mutuals"] if self.use_mutuals == 1 else None
        idx_1 = str(curr_file.split("_")[-2])
        idx_2 = str(curr_file.split("_")[-1].split(".")[0])
        scene = curr_file.split("/")[-2]

        def xyz(i):
            with np.load(os.path.join(self.root, "features", scene, scene + "_{}.npz".format(i)),
                         allow_pickle=False) as f:
                return f["xyz"]
        if mutuals is not None:
            xs = xs[mutuals.astype(bool).reshape(-1), :]
        return {"xs": np.expand_dims(xs, 0), "metadata": [scene, idx_1, idx_2], "idx": np.array(idx),
                "xyz1": [xyz(idx_1)], "xyz2": [xyz(idx_2)]}

    def __len__(self):
        return len(self.files)


def make_pairwise_eval_data_loader(args, num_workers=4, world=1, rank=0):
    """scripts/utils.py:146-197: the loader (batch 1 with mutuals, else args.batch_size; no shuffling) and
    scene_info {scene: [4 * first pair, 4 * end pair]} (row ranges of the stacked 4x4 estimates).

    world > 1: the loader covers only this rank's contiguous block of the evaluation's
    file list, made of whole loader batches (lib.distributed.shard_pairs with group = the batch size), so every
    batch — and with it the train-mode BatchNorm statistics and the zero-row guard of its forward — is exactly one
    of the single-process loader's batches.  Samples keep their global index ('idx').  `loader.pair_block` =
    [first, end) of this rank's block; scene_info always describes the whole evaluation."""
    from lib.distributed import shard_pairs
    dset = PrecomputedPairwiseEvalDataset(args)
    batch_size = 1 if args.mutuals else args.batch_size
    scene_info, nr = {}, 0
    for scene, files in _scene_files(args):
        scene_info[scene] = [nr * 4, (nr + len(files)) * 4]
        nr += len(files)
    scene_info["nr_examples"] = nr
    s, e = shard_pairs(len(dset), world, rank, group=batch_size)
    part = dset if (s, e) == (0, len(dset)) else data.Subset(dset, range(s, e))
    loader = torch.utils.data.DataLoader(part, batch_size=batch_size, shuffle=False, num_workers=num_workers,
                                         collate_fn=collate_fn, pin_memory=False, drop_last=False)
    loader.pair_block = (s, e)
    return loader, scene_info
