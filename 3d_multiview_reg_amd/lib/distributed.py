"""Multi-GPU sharding of the pair batch.

One process per GPU (torchrun; backend "nccl" = RCCL over xGMI on MI355X, "gloo" for the CPU
tests).  Pairs are independent given the fragment descriptors, so the only exchange is one
all-gather of fixed-size per-pair records at the end:

  * every rank computes the FCGF descriptors and samples of all fragments of the scene
    (cheap, and identical on every rank: same seeds), or receives them precomputed;
  * the lexicographic pair list (lib/utils.py:873 ``itertools.combinations``) is split into
    contiguous blocks of whole 32-pair groups (the reference evaluation batch,
    scripts/benchmark_pairwise_registration.py:363-367), so the batch-coupled zero-row guard of
    OANBlock (lib/filtering/oanet.py:177-178) sees exactly the reference's groups;
  * each rank runs Soft_NN -> OANet -> Procrustes on its block and packs one record per pair;
  * ``gather_records`` all-gathers the blocks (one collective, ~64 B per pair) into pair order.

Guard scope.  The reference evaluates the zero-row guard of OANBlock over its forward batch: 32 pairs in the
benchmark's loader batches ("group" mode, above: groups never straddle ranks, no exchange), but ALL pairs of a
scene when PairwiseReg.forward registers a whole scene at once (config 3).  "scene" mode reproduces the latter
across ranks: each block stops at its output head, one all-reduce (MAX) of the "some pair of mine has no positive
weight" bit over the ranks tells every rank whether the guard fires, and each rank then runs the block's
Procrustes on its own pairs (lib.filtering.oanet.OANet.guard_sync) — two 4-byte all-reduces per forward.
"""
import math

import numpy as np
import torch

GROUP = 32          # reference evaluation batch: the zero-row guard is evaluated per group
REC = 16            # floats per record: idx | R (9) | t (3) | conf | flag | pad


def shard_pairs(P, world, rank, group=GROUP):
    """Contiguous [start, end) block of the P pairs for `rank`, made of whole `group`-sized groups.
    Blocks are as equal as the grouping allows; trailing ranks may get an empty block."""
    if not 0 <= rank < world:
        raise ValueError("rank %d outside world %d" % (rank, world))
    n_groups = math.ceil(P / group)
    per = math.ceil(n_groups / world) if n_groups else 0
    g0 = min(rank * per, n_groups)
    g1 = min(g0 + per, n_groups)
    return min(g0 * group, P), min(g1 * group, P)


def block_capacity(P, world, group=GROUP):
    """Rows of the (equal-size, padded) per-rank block exchanged by gather_records."""
    n_groups = math.ceil(P / group)
    return (math.ceil(n_groups / world) if n_groups else 0) * group


def pack_records(first_pair, R, t, scores, flag=None):
    """Per-pair records [n, 16] float32: pair index, R row-major, t, conf = mean(scores > 0.5)
    (not a reference quantity), SVD-fallback flag."""
    n = R.shape[0]
    rec = torch.zeros(n, REC, dtype=torch.float32, device=R.device)
    rec[:, 0] = torch.arange(first_pair, first_pair + n, device=R.device, dtype=torch.float32)
    rec[:, 1:10] = R.reshape(n, 9).float()
    rec[:, 10:13] = t.reshape(n, 3).float()
    rec[:, 13] = (scores > 0.5).float().mean(dim=1)
    if flag is not None:
        flag = getattr(flag, "tensor", flag)   # lib.filtering.oanet.DeviceFlag: stays on the device
        rec[:, 14] = torch.as_tensor(flag, device=R.device).float().reshape(-1).expand(n)
    return rec


def _host_staged(pg=None):
    """gloo moves host tensors only: device tensors are staged through host memory (the CPU tests and the
    several-ranks-on-one-GPU rehearsal run gloo; RCCL takes device tensors directly)."""
    import torch.distributed as dist
    return dist.get_backend(pg) == "gloo"


def all_reduce_max(t, pg=None):
    """in-place MAX all-reduce of a small tensor (host-staged under gloo)"""
    import torch.distributed as dist
    if _host_staged(pg) and t.device.type != "cpu":
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.MAX, group=pg)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=pg)
    return t


def all_gather_rows(buf, world, pg=None):
    """[world * rows, ...] = every rank's equal-shape `buf` in rank order (host-staged under gloo)"""
    import torch.distributed as dist
    if _host_staged(pg):
        h = buf.cpu()
        parts = [torch.empty_like(h) for _ in range(world)]
        dist.all_gather(parts, h, group=pg)
        return torch.cat(parts).to(buf.device)
    out = torch.empty((world * buf.shape[0],) + tuple(buf.shape[1:]), dtype=buf.dtype, device=buf.device)
    dist.all_gather_into_tensor(out, buf.contiguous(), group=pg)
    return out


def gather_records(rec, P, world, group=GROUP, pg=None):
    """All-gather every rank's block of records (padded to block_capacity rows) and return the
    [P, width] records of all pairs in pair order, on every rank.  Any record width and dtype (the evaluation
    harness gathers float64 rows: its estimates are written to traj.txt in full precision)."""
    if world == 1:
        return rec
    cap = block_capacity(P, world, group)
    buf = torch.zeros((cap,) + tuple(rec.shape[1:]), dtype=rec.dtype, device=rec.device)
    buf[:rec.shape[0]] = rec
    out = all_gather_rows(buf, world, pg)
    rows = []
    for r in range(world):
        s, e = shard_pairs(P, world, r, group)
        rows.append(out[r * cap:r * cap + (e - s)])
    return torch.cat(rows)


def init_from_env(backend=None):
    """torchrun's environment (WORLD_SIZE / RANK / LOCAL_RANK / MASTER_*) -> (world, rank, device).
    WORLD_SIZE > 1 initialises the default process group once: backend "nccl" (RCCL over xGMI) when a HIP device
    is present, else "gloo"; under gloo several ranks may share the box's GPUs (LOCAL_RANK modulo the device
    count).  A world of one needs no process group."""
    import os
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    has_gpu = torch.cuda.is_available()
    backend = backend or ("nccl" if has_gpu else "gloo")
    dev = torch.device("cpu")
    if has_gpu:
        if backend != "nccl":
            local %= max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    return world, rank, dev


def collective_device(pg=None):
    """where a collective's tensors live: the current HIP device under RCCL, the host under gloo"""
    import torch.distributed as dist
    if dist.get_backend(pg) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def unpack_records(rec):
    """-> (pair_idx int64 [P], R [P,3,3], t [P,3,1], conf [P], flag bool [P]) on the host."""
    a = rec.detach().cpu().numpy()
    return (a[:, 0].astype(np.int64), a[:, 1:10].reshape(-1, 3, 3), a[:, 10:13].reshape(-1, 3, 1), a[:, 13],
            a[:, 14] > 0)


def scene_guard_sync(world, pg=None):
    """guard_sync for OANet (lib.filtering.oanet.OANet.guard_sync): the zero-row guard over the pairs of every
    rank.  guard_pos [p] int32 (positive weights per local pair) -> counts that fire the local guard exactly when
    some pair on SOME rank has none: one all-reduce (MAX) of the local bit, no host synchronisation (RCCL).
    The returned counts only steer the guard (mvr_procrustes tests them for a zero and uses them for nothing
    else), so forcing the first one to 0 fires it for every local pair."""
    def sync(guard_pos):
        bit = (guard_pos == 0).any().to(torch.int32).reshape(1) if guard_pos.numel() else \
            torch.zeros(1, dtype=torch.int32, device=guard_pos.device)
        if world > 1:
            all_reduce_max(bit, pg)
        if guard_pos.numel() == 0:
            return guard_pos
        g = guard_pos.clone()
        g[:1] = torch.where(bit > 0, torch.zeros_like(g[:1]), g[:1])   # a zero count fires the whole local batch
        return g
    return sync


def register_pairs_sharded(model, filtering_input, world, rank, group=GROUP, guard="group", pg=None,
                           first_pair=None):
    """Run model.filter_correspondences on this rank's block of the pair batch and all-gather the records.
    guard="group": the zero-row guard evaluated per `group` pairs (the reference's batch-32 evaluation), and in
    train mode the BatchNorm batch statistics per `group` pairs too (the benchmark's 32-pair loader batches,
    scripts/benchmark_pairwise_registration.py:159-197, which never calls model.eval());
    guard="scene": over the whole batch of all ranks (the reference's PairwiseReg.forward over a scene, eval mode:
    train-mode statistics over a batch split across ranks would need an exchange of BatchNorm moments, which
    this path does not do, so it raises).
    `filtering_input` is the dict of lib/utils.py:construct_filtering_input_data over ALL pairs (every rank
    holds it), or — with first_pair given — only this rank's block [first_pair, first_pair + n) of a batch of
    filtering_input["num_pairs"] pairs (the bench's pair-sharded scene: each rank matches its own block)."""
    if guard not in ("group", "scene"):
        raise ValueError(guard)
    xs = filtering_input["xs"]
    if first_pair is None:
        P = xs.shape[0]
        s, e = shard_pairs(P, world, rank, group)
        xs_mine = xs[s:e]
    else:
        P = int(filtering_input["num_pairs"])
        s, e = shard_pairs(P, world, rank, group)
        if (s, e) != (first_pair, first_pair + xs.shape[0]):
            raise ValueError("block [%d, %d) is not rank %d's shard [%d, %d)" % (first_pair, first_pair + xs.shape[0],
                                                                                rank, s, e))
        xs_mine = xs
    filt = model.filtering_module if hasattr(model, "filtering_module") else model
    if guard == "scene" and filt.training:
        raise ValueError("guard='scene' shards an eval-mode forward (train-mode BatchNorm statistics would span ranks)")
    sync = scene_guard_sync(world, pg) if guard == "scene" else None
    if e > s:
        prev = (filt.guard_group, filt.guard_sync, getattr(filt, "bn_group", 0))
        filt.guard_group, filt.guard_sync = (group, None) if guard == "group" else (0, sync)
        filt.bn_group = group if guard == "group" else 0
        try:
            out = model.filter_correspondences({"xs": xs_mine}) if hasattr(model, "filter_correspondences") \
                else model({"xs": xs_mine})
        finally:
            filt.guard_group, filt.guard_sync, filt.bn_group = prev
        rec = pack_records(s, out["rot_est"][-1], out["trans_est"][-1], out["scores"][-1],
                           out.get("gradient_flag"))
    else:
        if sync is not None:   # an empty block still takes part in every block's all-reduce
            for _ in range(1 + getattr(filt, "iter_num", 0)):
                sync(torch.zeros(0, dtype=torch.int32, device=xs.device))
        rec = torch.zeros(0, REC, device=xs.device)
    return gather_records(rec, P, world, group, pg)
