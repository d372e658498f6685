"""Pair-batch sharding across ranks (lib/distributed.py) on CPU with the gloo
backend, world size 2: contiguous 32-pair-aligned blocks, one all-gather of records, results
in pair order identical to the single-rank run, guard groups aligned with the reference batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lib import distributed as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("P", [0, 1, 31, 32, 33, 435, 1000])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_pairs_partition(P, world):
    blocks = [D.shard_pairs(P, world, r) for r in range(world)]
    assert blocks[0][0] == 0 and blocks[-1][1] == P
    for (s0, e0), (s1, e1) in zip(blocks, blocks[1:]):
        assert e0 == s1                        # contiguous, disjoint, in rank order
    cap = D.block_capacity(P, world)
    for s, e in blocks:
        assert e == s or s % D.GROUP == 0     # guard groups never straddle two ranks
        assert 0 <= e - s <= cap


class _StubFilter(torch.nn.Module):
    """Deterministic per-pair stand-in for PairwiseReg.filter_correspondences (CPU) with the reference's
    batch-coupled zero-row guard (oanet.py:177-178): weights relu(x0) per point; if some pair of the guard's scope
    has no positive weight, every pair of that scope gets + 1/N; R, t from the weighted means.  The guard's scope
    follows the OANet contract: guard_sync (scene mode: the whole sharded batch), else guard_group (> 0: groups of
    that many pairs), else the whole forward batch."""

    iter_num = 0

    def __init__(self):
        super().__init__()
        self.eval()                      # scene mode shards eval-mode forwards only
        self.guard_group = 0
        self.guard_sync = None
        self.seen = []

    def filter_correspondences(self, d):
        xs = d["xs"][:, 0]                                          # [p, N, 6]
        self.seen.append((self.guard_group, self.guard_sync is not None))
        p, n = xs.shape[:2]
        w = torch.relu(xs[..., 0])
        pos = (w > 0).sum(dim=1).to(torch.int32)
        if self.guard_sync is not None:
            fire = torch.full((p,), bool((self.guard_sync(pos) == 0).any()))
        else:
            g = self.guard_group if self.guard_group > 0 else max(p, 1)
            grp = torch.arange(p) // g
            zero = (pos == 0)
            fire = torch.stack([zero[grp == k].any() for k in grp.tolist()]) if p else torch.zeros(0, dtype=torch.bool)
        w = w + fire[:, None].float() / n
        wn = w / (w.sum(dim=1, keepdim=True) + 1e-7)
        m = (wn[..., None] * xs).sum(dim=1)                          # [p, 6]
        R = torch.eye(3).repeat(p, 1, 1) + m[:, :3, None] * 1e-3
        t = m[:, 3:6, None]
        return {"rot_est": [R], "trans_est": [t], "scores": [w], "gradient_flag": False}


def _xs(P, N=16, zero_pair=None):
    g = torch.Generator().manual_seed(5)
    xs = torch.randn(P, 1, N, 6, generator=g)
    if zero_pair is not None and zero_pair < P:
        xs[zero_pair, 0, :, 0] = -xs[zero_pair, 0, :, 0].abs() - 0.1   # no positive weight: the guard fires
    return xs


def _worker(rank, world, port, P, guard, zero_pair, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        stub = _StubFilter()
        rec = D.register_pairs_sharded(stub, {"xs": _xs(P, zero_pair=zero_pair)}, world, rank, guard=guard)
        # the raw gather of hand-made records, too
        s, e = D.shard_pairs(P, world, rank)
        mine = torch.arange(s, e, dtype=torch.float32)[:, None].repeat(1, D.REC)
        g = D.gather_records(mine, P, world)
        q.put((rank, rec.numpy(), g.numpy(), (stub.guard_group, stub.guard_sync), stub.seen))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P,guard,zero_pair", [(70, "group", None), (435, "group", None), (70, "group", 66),
                                               (70, "scene", 66), (70, "scene", None), (40, "scene", 35)])
def test_register_sharded_gloo_world2(P, guard, zero_pair):
    """world 2 reproduces the single-rank records exactly, in pair order.  With a zero-weight pair on rank 1
    (pair 66 of 70: rank 0 holds pairs 0-63): "group" mode fires the guard in that pair's 32-pair group only,
    "scene" mode on every pair of both ranks (one all-reduce per block), as the single-rank run over the batch."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, guard, zero_pair, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = D.register_pairs_sharded(_StubFilter(), {"xs": _xs(P, zero_pair=zero_pair)}, 1, 0, guard=guard).numpy()
    for rank, rec, g, restored, seen in res:
        assert rec.shape == (P, D.REC)
        np.testing.assert_array_equal(rec[:, 0], np.arange(P))        # pair order
        np.testing.assert_allclose(rec, ref, rtol=0, atol=0)           # identical to one rank
        np.testing.assert_array_equal(g[:, 0], np.arange(P))
        assert restored == (0, None)                                   # guard scope set, then restored
        if seen:
            assert all(x == ((D.GROUP, False) if guard == "group" else (0, True)) for x in seen)
    if zero_pair is not None:
        # the guard's reach: every pair (scene) or the zero pair's 32-pair group only (group)
        plain = D.register_pairs_sharded(_StubFilter(), {"xs": _xs(P)}, 1, 0, guard=guard).numpy()
        hit = np.any(ref != plain, axis=1)
        if guard == "scene":
            assert hit.all()
        else:
            grp = np.arange(P) // D.GROUP
            np.testing.assert_array_equal(hit, grp == zero_pair // D.GROUP)


def test_pack_unpack_roundtrip():
    R = torch.randn(5, 3, 3)
    t = torch.randn(5, 3, 1)
    sc = torch.rand(5, 100)
    idx, R2, t2, conf, flag = D.unpack_records(D.pack_records(7, R, t, sc, True))
    np.testing.assert_array_equal(idx, np.arange(7, 12))
    np.testing.assert_allclose(R2, R.numpy())
    np.testing.assert_allclose(t2, t.numpy())
    np.testing.assert_allclose(conf, (sc > 0.5).float().mean(1).numpy())
    assert flag.all()


def _worker_own_block(rank, world, port, P, q):
    """each rank holds only its own block of the filtering input (the bench's pair-sharded scene: a rank matches
    only its pairs) and says where it starts"""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, e = D.shard_pairs(P, world, rank, group=1)
        xs = _xs(P, zero_pair=P - 3)[s:e]
        rec = D.register_pairs_sharded(_StubFilter(), {"xs": xs, "num_pairs": P}, world, rank, group=1,
                                       guard="scene", first_pair=s)
        q.put((rank, rec.numpy()))
    finally:
        dist.destroy_process_group()


def test_register_sharded_own_block_gloo_world2():
    """first_pair mode (the input holds only this rank's block, balanced single-pair groups): the gathered records
    equal one rank over the whole batch, the scene guard firing from the last rank's zero pair"""
    P, world = 45, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_own_block, args=(r, world, port, P, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = D.register_pairs_sharded(_StubFilter(), {"xs": _xs(P, zero_pair=P - 3)}, 1, 0, group=1, guard="scene").numpy()
    for _, rec in res:
        np.testing.assert_array_equal(rec, ref)


def test_register_sharded_contract_errors():
    """scene guard over a train-mode (batch-statistics) forward would need the BatchNorm moments of every rank:
    refused; a block that is not the rank's shard: refused"""
    stub = _StubFilter()
    stub.train()
    with pytest.raises(ValueError):
        D.register_pairs_sharded(stub, {"xs": _xs(8)}, 1, 0, guard="scene")
    stub.eval()
    with pytest.raises(ValueError):
        D.register_pairs_sharded(stub, {"xs": _xs(8)[:5], "num_pairs": 8}, 1, 0, guard="scene", first_pair=2)


def test_register_sharded_group_mode_sets_bn_groups():
    """group mode runs the filter with guard and BatchNorm groups of `group` pairs (the benchmark's loader
    batches) and restores the filter's settings afterwards"""
    class Spy(_StubFilter):
        def filter_correspondences(self, d):
            self.during = (self.guard_group, self.bn_group)
            return super().filter_correspondences(d)
    s = Spy()
    s.bn_group = 0
    D.register_pairs_sharded(s, {"xs": _xs(40)}, 1, 0, guard="group")
    assert s.during == (D.GROUP, D.GROUP)
    assert (s.guard_group, s.bn_group) == (0, 0)
