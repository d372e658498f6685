"""Pairwise registration benchmark on precomputed correspondences (3DMatch / Redwood layout).

Mirrors scripts/benchmark_pairwise_registration.py of the reference (same CLI flags, result files and
report), with the per-pair host loop replaced by batched GPU calls:
  * method RegBlock / any filtering config: `PairwiseReg.filter_correspondences` on each loader batch
    (OANet + Procrustes on the GPU, benchmark:195-216), `--refine` = batched GPU RANSAC over each pair's
    inliers (scores > 0.5, benchmark:209-212);
  * method RANSAC: batched GPU RANSAC over all correspondences of a batch (benchmark:56-133);
  * T_est = inv(estimate), overlap flag = compute_overlap_ratio(xyz1, xyz2, T_est) >= 0.3 (3DMatch) / 0.23
    (Redwood) on the GPU (lib/overlap.py; every pair of a loader batch in one FragmentOverlap.ratios call),
    trajectories written per scene (benchmark:222-245, with the
    bool-flag fix of lib/utils.py write_trajectory), then precision / recall / rotation and translation
    errors per scene against gt.log / gt.info (benchmark:250-345).
Optional reference dependencies that are absent here (open3d, coloredlogs, matplotlib) are not needed.
A run without --model uses random-init weights (no checkpoint download offline) and says so.

usage (from a directory holding configs/pairwise_registration/eval/<method>.yaml, or with --config):
  python -m scripts.benchmark_pairwise_registration --source_path ./data/eval_data/ --dataset 3d_match \
      --method RegBlock --model ./pretrained/RegBlock/model_best.pt [--refine] [--mutuals] [--only_gt_overlaping]
"""
import argparse
import logging
import os
import sys
from collections import defaultdict

import numpy as np
import torch

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from lib.utils import (ensure_dir, read_trajectory, write_trajectory, read_trajectory_info,  # noqa: E402
                       get_folder_list, Timer, rotation_error, translation_error, load_config,
                       evaluate_registration, extract_corresponding_trajectors,
                       run_ransac_batch)
from scripts.utils import make_pairwise_eval_data_loader  # noqa: E402
from lib.checkpoints import CheckpointIO  # noqa: E402
from lib.overlap import FragmentOverlap  # noqa: E402
import lib.config as config  # noqa: E402

SHORT_NAMES = {
    "3d_match": {"kitchen": "Kitchen", "sun3d-home_at-home_at_scan1_2013_jan_1": "Home 1",
                 "sun3d-home_md-home_md_scan9_2012_sep_30": "Home 2", "sun3d-hotel_uc-scan3": "Hotel 1",
                 "sun3d-hotel_umd-maryland_hotel1": "Hotel 2", "sun3d-hotel_umd-maryland_hotel3": "Hotel 3",
                 "sun3d-mit_76_studyroom-76-1studyroom2": "Study",
                 "sun3d-mit_lab_hj-lab_hj_tea_nov_2_2012_scan1_erika": "MIT Lab"},
    "redwood": {"iclnuim-livingroom1": "livingroom1", "iclnuim-livingroom2": "livingroom2",
                "iclnuim-office1": "office1", "iclnuim-office2": "office2"}}


def _save_path(source_path, method, mutuals):
    return os.path.join(source_path, "results", method) + ("/mutuals/" if mutuals else "/all/")


def _ransac(xs, keep=None, seed=0):
    """batched RANSAC over [B, N, 6] correspondences (rows where `keep`, in their original order)"""
    xs = np.asarray(xs, np.float64)
    if keep is None:
        return run_ransac_batch(xs[..., :3], xs[..., 3:], seed=seed)
    order = np.argsort(~keep, axis=1, kind="stable")
    x = np.take_along_axis(xs, order[..., None], axis=1)
    return run_ransac_batch(x[..., :3], x[..., 3:], counts=keep.sum(1), seed=seed)


def load_model(method, model_path, cfg_path=None):
    """benchmark:155-169: the method's YAML, read with load_config exactly as the reference does (a missing file
    is an error there and here), then lib.config.get_model and the optional checkpoint"""
    cfg_path = cfg_path or os.path.join("./configs/pairwise_registration/eval", method + ".yaml")
    cfg = load_config(cfg_path)
    model = config.get_model(cfg)
    if model_path:
        ckpt = CheckpointIO("/".join(model_path.split("/")[0:-1]), initialize_from=None,
                            initialization_file_name=None, model=model)
        ckpt.load(model_path.split("/")[-1])
    else:
        logging.warning("no --model given: random-init weights (registration quality is meaningless)")
    return model.to(torch.device("cuda"))


# per-pair record of the estimation loop: [pair idx, T_est (4 x 4, row-major), overlap flag, fragment i, fragment j]
REC = 20


def _batch_records(batch, bi, method, model, refine, seed, overlap_method, overlap_threshold):
    """benchmark:193-224 for one loader batch: the estimate of every pair (batched: OANet + Procrustes, or RANSAC,
    on the GPU), T_est = inv(estimate), the overlap gate -> float64 records [b, REC].  `bi` is the batch's index
    in the whole evaluation (it seeds the RANSAC draws, so a batch gets the same draws on whichever rank it runs)."""
    xs = batch["xs"][:, 0].numpy()
    if method == "RANSAC":
        T = _ransac(xs, seed=seed + bi)
    else:
        out = model.filter_correspondences(batch)
        R = out["rot_est"][-1].double().cpu().numpy()
        t = out["trans_est"][-1].double().cpu().numpy().reshape(-1, 3)
        if refine:
            T = _ransac(xs, keep=out["scores"][-1].cpu().numpy() > 0.5, seed=seed + bi)
        else:
            T = np.tile(np.eye(4), (len(R), 1, 1))
            T[:, :3, :3], T[:, :3, 3] = R, t
    # the overlap gate of every pair of the batch in one call (benchmark:217-220 scores one pair at a time on
    # the CPU): the batch's 2B clouds indexed once on the GPU, pair k = clouds (2k, 2k + 1)
    T_est = np.linalg.inv(T)
    b = T.shape[0]
    clouds = [c for k in range(b) for c in (batch["xyz1"][k][0], batch["xyz2"][k][0])]
    ratios = FragmentOverlap(clouds, method=overlap_method).ratios(
        [[2 * k, 2 * k + 1] for k in range(b)], list(T_est)) if b else []
    rec = np.zeros((b, REC), np.float64)
    for k in range(b):
        meta = batch["metadata"][k]
        rec[k, 0] = int(batch["idx"][k].numpy().item())
        rec[k, 1:17] = T_est[k].reshape(16)
        rec[k, 17] = float(ratios[k] >= overlap_threshold)
        rec[k, 18], rec[k, 19] = int(meta[1]), int(meta[2])
    return rec


def _gather_records(rec, num_pairs, batch_size, world, pg=None):
    """every rank's records -> the records of all pairs in pair order (one all-gather over RCCL, ~160 B per pair;
    host-staged under gloo): lib.distributed.gather_records over the loader's batch-aligned blocks"""
    if world == 1:
        return rec
    from lib import distributed as D
    dev = D.collective_device(pg)
    out = D.gather_records(torch.from_numpy(rec).to(dev), num_pairs, world, group=batch_size, pg=pg)
    return out.cpu().numpy()


def estimate_trans_params(eval_data, source_path, dataset, scene_info, method, model, mutuals,
                          overlap_method="FCGF", refine=False, seed=0, world=1, rank=0):
    """benchmark:56-133 (method RANSAC) and :137-245 (learned filters), batched: writes traj.txt per scene.
    world > 1: `eval_data` is this rank's block of whole loader batches (lib.data.make_pairwise_eval_data_loader);
    the per-pair records are all-gathered and rank 0 writes the trajectories."""
    num_pairs = scene_info["nr_examples"]
    est = np.tile(np.eye(4), reps=[num_pairs, 1])
    save_path = _save_path(source_path, method, mutuals)
    overlap_threshold = 0.3 if dataset == "3d_match" else 0.23
    logging.info("Starting %s based registration estimation for %d pairs (overlap threshold %.2f, %d rank%s)!",
                 method, num_pairs, overlap_threshold, world, "s" if world > 1 else "")
    first = getattr(eval_data, "pair_block", (0, num_pairs))[0]
    bsz = eval_data.batch_size or 1
    timer, full = Timer(), Timer()
    full.tic()
    recs = []
    for bi, batch in enumerate(eval_data):
        timer.tic()
        recs.append(_batch_records(batch, first // bsz + bi, method, model, refine, seed, overlap_method,
                                   overlap_threshold))
        timer.toc()
    rec = np.concatenate(recs) if recs else np.zeros((0, REC), np.float64)
    rec = _gather_records(rec, num_pairs, bsz, world)
    if num_pairs and recs:
        logging.info("%d pairwise registration parameters estimated in %.3fs (%.4fs per batch of pure run time)",
                     num_pairs, full.toc(average=False), timer.avg)
    if rank != 0:
        return
    order = np.argsort(rec[:, 0], kind="stable")
    rec = rec[order]
    assert rec.shape[0] == num_pairs and np.array_equal(rec[:, 0], np.arange(num_pairs)), "records of every pair"
    reg_metadata = []
    for r in rec:
        p = int(r[0])
        est[4 * p:4 * p + 4, :] = r[1:17].reshape(4, 4)
        reg_metadata.append([str(int(r[18])), str(int(r[19])), bool(r[17])])
    ensure_dir(save_path)
    for key, rng in scene_info.items():
        if key == "nr_examples":
            continue
        ensure_dir(os.path.join(save_path, key))
        write_trajectory(est[rng[0]:rng[1], :].reshape(-1, 4, 4), reg_metadata[rng[0] // 4:rng[1] // 4],
                         os.path.join(save_path, key, "traj.txt"))


def evaluate_registration_performance(eval_data, source_path, dataset, scene_info, method, model, mutuals=False,
                                      overlap_method="FCGF", refine=False, seed=0, world=1, rank=0):
    """benchmark:250-345: estimate (scenes without results), then the per-scene report; returns the summary.
    world > 1: rank 0 writes the trajectories and the report; every rank returns rank 0's summary."""
    estimate_trans_params(eval_data, source_path, dataset, scene_info, method, model, mutuals, overlap_method,
                          refine, seed, world, rank)
    if world > 1:
        import torch.distributed as dist
        box = [_report(source_path, dataset, method, mutuals) if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        return box[0]
    return _report(source_path, dataset, method, mutuals)


def _report(source_path, dataset, method, mutuals):
    """benchmark:280-345: precision / recall / rotation and translation errors per scene against gt.log / gt.info"""
    re_medians, te_medians, precision, recall = [], [], [], []
    per_scene = {}
    logging.info("Results of %s on %s dataset!", method, dataset)
    logging.info("%-12s | prec. | rec.  |   re  |   te  |", "Scene")
    for folder in get_folder_list(os.path.join(source_path, "correspondences")):
        scene = folder.split("/")[-1]
        gt_pairs, gt_traj = read_trajectory(os.path.join(source_path, "raw_data", scene, "gt.log"))
        n_fragments, gt_cov = read_trajectory_info(os.path.join(source_path, "raw_data", scene, "gt.info"))
        assert gt_traj.shape[0] > 0, "Empty trajectory file"
        est_pairs, est_traj = read_trajectory(os.path.join(_save_path(source_path, method, mutuals), scene,
                                                           "traj.txt"))
        if est_traj.shape[0] == 0:
            p, r, re, te = 0.0, 0.0, np.array([np.nan]), np.array([np.nan])
        else:
            p, r = evaluate_registration(n_fragments, est_traj, est_pairs, gt_pairs, gt_traj, gt_cov)
            e_est, e_gt = extract_corresponding_trajectors(est_pairs, gt_pairs, est_traj, gt_traj)
            re = rotation_error(torch.from_numpy(e_gt[:, 0:3, 0:3]), torch.from_numpy(e_est[:, 0:3, 0:3])).numpy()
            te = translation_error(torch.from_numpy(e_gt[:, 0:3, 3:4]), torch.from_numpy(e_est[:, 0:3, 3:4])).numpy()
        precision.append(p)
        recall.append(r)
        re_medians.append(np.median(re))
        te_medians.append(np.median(te))
        per_scene[scene] = (p, r, float(np.median(re)), float(np.median(te)))
        logging.info("%-12s | %.3f | %.3f | %.3f | %.3f |", SHORT_NAMES.get(dataset, {}).get(scene, scene)[:12],
                     p, r, np.median(re), np.median(te))
    summary = {"precision": float(np.mean(precision)), "recall": float(np.mean(recall)),
               "re": float(np.mean(re_medians)), "te": float(np.mean(te_medians)), "scenes": per_scene}
    logging.info("Mean precision: %.3f +- %.3f", np.mean(precision), np.std(precision))
    logging.info("Mean recall: %.3f +- %.3f", np.mean(recall), np.std(recall))
    logging.info("Mean ae: %.3f +- %.3f [deg]", np.mean(re_medians), np.std(re_medians))
    logging.info("Mean te: %.3f +- %.3f [m]", np.mean(te_medians), np.std(te_medians))
    return summary


def parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--source_path", default="./data/eval_data/", type=str, help="path to dataset")
    ap.add_argument("--dataset", default="3d_match", type=str, help="dataset [3d_match, redwood]")
    ap.add_argument("--method", default="OANet", type=str, help="Which method should be used [RANSAC, RegBlock, Joint]")
    ap.add_argument("--model", default=None, type=str, help="path to latest checkpoint (default: None)")
    ap.add_argument("--batch_size", type=int, default=32, help="Batch size (if mutuals are selected batch size will be 1).")
    ap.add_argument("--mutuals", action="store_true", help="If only mutually closest NN should be used (reciprocal matching).")
    ap.add_argument("--save_data", action="store_true", help="(accepted for compatibility; not written)")
    ap.add_argument("--overwrite", action="store_true", help="Overwrite existing results of this method and dataset")
    ap.add_argument("--overlap_method", type=str, default="FCGF", help="Overlap ratio method (FCGF or 3DMatch)")
    ap.add_argument("--only_gt_overlaping", action="store_true", help="Only the GT overlapping pairs")
    ap.add_argument("--refine", action="store_true", help="RANSAC over the network's inliers")
    ap.add_argument("--config", default=None, type=str, help="filtering config YAML (default ./configs/pairwise_"
                    "registration/eval/<method>.yaml, as the reference reads it)")
    ap.add_argument("--seed", type=int, default=0, help="RANSAC draw stream seed")
    ap.add_argument("--num_workers", type=int, default=4)
    ap.add_argument("--dist_backend", default=None, choices=["nccl", "gloo"],
                    help="under torchrun (WORLD_SIZE > 1): the process group's backend (default nccl = RCCL on a GPU "
                    "box, gloo without one); the evaluation's file list is split into contiguous blocks of whole "
                    "batches over the ranks, the per-pair records all-gathered, the results written by rank 0")
    return ap


def main(argv=None):
    from lib.distributed import init_from_env
    args = parser().parse_args(argv)
    world, rank, _ = init_from_env(args.dist_backend)
    logging.basicConfig(level=logging.INFO if rank == 0 else logging.WARNING,
                        format="%(asctime)s [%(levelname)s] %(message)s")
    assert args.source_path is not None
    args.source_path = os.path.join(args.source_path, args.dataset)
    eval_data, scene_info = make_pairwise_eval_data_loader(args, num_workers=args.num_workers, world=world, rank=rank)
    model = None if args.method == "RANSAC" else load_model(args.method, args.model, args.config)
    with torch.no_grad():
        return evaluate_registration_performance(eval_data, args.source_path, args.dataset, scene_info, args.method,
                                                 model, args.mutuals, args.overlap_method, args.refine, args.seed,
                                                 world, rank)


if __name__ == "__main__":
    main()
