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
    """Deterministic per-pair stand-in for PairwiseReg.filter_correspondences (CPU): R, t and
    scores are functions of each pair's own xs, so sharding must not change them."""

    def __init__(self):
        super().__init__()
        self.guard_group = 0
        self.seen_groups = []

    def filter_correspondences(self, d):
        xs = d["xs"][:, 0]                                          # [p, N, 6]
        self.seen_groups.append(self.guard_group)
        m = xs.mean(dim=1)                                          # [p, 6]
        R = torch.eye(3).repeat(xs.shape[0], 1, 1) + m[:, :3, None] * 1e-3
        t = m[:, 3:6, None]
        scores = torch.sigmoid(xs[..., 0])
        return {"rot_est": [R], "trans_est": [t], "scores": [scores], "gradient_flag": False}


def _xs(P, N=16):
    g = torch.Generator().manual_seed(5)
    return torch.randn(P, 1, N, 6, generator=g)


def _worker(rank, world, port, P, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        stub = _StubFilter()
        rec = D.register_pairs_sharded(stub, {"xs": _xs(P)}, world, rank)
        # the raw gather of hand-made records, too
        s, e = D.shard_pairs(P, world, rank)
        mine = torch.arange(s, e, dtype=torch.float32)[:, None].repeat(1, D.REC)
        g = D.gather_records(mine, P, world)
        q.put((rank, rec.numpy(), g.numpy(), stub.guard_group, stub.seen_groups))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P", [70, 435])
def test_register_sharded_gloo_world2(P):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = D.register_pairs_sharded(_StubFilter(), {"xs": _xs(P)}, 1, 0)
    for rank, rec, g, gg, seen in res:
        assert rec.shape == (P, D.REC)
        np.testing.assert_array_equal(rec[:, 0], np.arange(P))        # pair order
        np.testing.assert_allclose(rec, ref.numpy(), rtol=0, atol=0)   # identical to one rank
        np.testing.assert_array_equal(g[:, 0], np.arange(P))
        assert gg == 0 and all(x == D.GROUP for x in seen)             # guard scope set, then restored


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
