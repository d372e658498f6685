"""Pairwise registration demo (scripts/pairwise_demo.py of the reference): two point clouds -> the relative
transformation, written to ./data/demo/pairwise/results/est_T.log.

Same CLI and output file as the reference; the whole chain runs on the GPU through the lib.* surface:
PLY read (lib/ply.py instead of open3d), voxelisation (lib.sparse.voxelize instead of ME.sparse_quantize,
pairwise_demo.py:61-98), PairwiseReg.compute_descriptors (FCGF -> sampling -> feature NN) and
filter_correspondences (OANet -> Procrustes).  --visualize needs open3d, which is absent: it is reported
and skipped.

usage: python -m scripts.pairwise_demo configs/pairwise_registration/demo/config.yaml \
           [--source_pc ...cloud_bin_0.ply] [--target_pc ...cloud_bin_1.ply] [--model pairwise_reg.pt] [--verbose]
"""
import argparse
import logging
import os
import sys
import time

import numpy as np
import torch

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

import lib.config as config  # noqa: E402
from lib.checkpoints import CheckpointIO  # noqa: E402
from lib.ply import read_ply_xyz  # noqa: E402
from lib.sparse import voxelize  # noqa: E402
from lib.utils import load_config, write_trajectory  # noqa: E402


def prepare_data(point_cloud_files, voxel_size, device):
    """pairwise_demo.py:61-98: voxel-downsampled clouds + the batched sparse input of FCGF"""
    raw = [read_ply_xyz(f) for f in point_cloud_files]
    coords, _, counts, xyz_down = voxelize(raw, voxel_size, device)
    return {"pcd0": xyz_down, "sinput0_C": coords, "sinput0_F": torch.ones(coords.shape[0], 1, device=device),
            "pts_list": torch.tensor(counts)}


def main(cfg, args, logger=logging.getLogger()):
    np.random.seed(41)     # pairwise_demo.py:25-28 (the Sampler draws on numpy's global RandomState)
    torch.manual_seed(41)
    model = config.get_model(cfg)
    model.eval()
    ckpt = CheckpointIO("", initialize_from="./pretrained/", initialization_file_name=args.model, model=model)
    try:
        ckpt.load()
    except FileExistsError:
        logger.warning("no pretrained model %s: random-init weights", args.model)
    logger.info("Total number of model parameters: %d", sum(p.numel() for p in model.parameters()))
    target_base = "./data/demo/pairwise/results"
    id_0 = args.source_pc.split(os.sep)[-1].split("_")[-1].split(".")[0]
    id_1 = args.target_pc.split(os.sep)[-1].split("_")[-1].split(".")[0]
    os.makedirs(target_base, exist_ok=True)
    target_path = os.path.join(target_base, "est_T.log")
    dev = torch.device("cuda")
    with torch.no_grad():
        t0 = time.time()
        data = prepare_data([args.source_pc, args.target_pc], cfg["misc"]["voxel_size"], dev)
        t1 = time.time()
        filtering_data, _, _ = model.compute_descriptors(data)
        t2 = time.time()
        est = model.filter_correspondences(filtering_data)
        est_T = np.eye(4)
        est_T[0:3, 0:3] = est["rot_est"][-1].cpu().numpy()
        est_T[0:3, 3:4] = est["trans_est"][-1].cpu().numpy()
        t3 = time.time()
    write_trajectory(np.expand_dims(est_T, 0), [[id_0, id_1, "True"]], target_path)
    if args.verbose:
        logger.info("Feature computation and sampling took %.3fs", t2 - t1)
        logger.info("Filtering the correspondences and estimation of paramaters took %.3fs", t3 - t2)
        logger.info("Estimation of the pairwise transformation parameters completed in %.3fs", t3 - t0)
        logger.info("Estimated parameters were saved in %s.", target_path)
    if args.visualize:
        logger.warning("--visualize needs open3d (not available): skipped")
    return est_T


def parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", default="./configs/pairwise_registration/demo/config.yaml", type=str, help="config file")
    ap.add_argument("--source_pc", default="./data/demo/pairwise/raw_data/cloud_bin_0.ply", type=str)
    ap.add_argument("--target_pc", default="./data/demo/pairwise/raw_data/cloud_bin_1.ply", type=str)
    ap.add_argument("--model", default="pairwise_reg.pt", type=str, help="Name of the pretrained model.")
    ap.add_argument("--verbose", action="store_true", help="Write out the intermediate results and timings")
    ap.add_argument("--visualize", action="store_true", help="Visualize the point cloud and the results.")
    return ap


if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO, format="%(asctime)s [%(levelname)s] %(name)s - %(message)s")
    a = parser().parse_args()
    main(load_config(a.config), a)
