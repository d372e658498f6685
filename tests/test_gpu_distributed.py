"""The pair-sharded path (lib/distributed.py) with the REAL HIP filter in several processes: two
ranks on the box's one GPU (gloo, collectives staged through host memory; RCCL refuses two ranks on one device),
each running OANet (RegBlock size) + Procrustes on its block of 70 pairs.  The zero-row guard
(lib/filtering/oanet.py:177-178) fires for pairs that all live on rank 0; the gathered records must be
bit-identical to one process over the whole batch — in scene mode (eval, the guard over all pairs of both ranks:
rank 1's pairs get + 1/N although none of them has a zero row) and in group mode (train-mode BatchNorm and the
guard per 32-pair group, the benchmark's loader batches)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "helpers", "dist_worker.py")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("guard", ["scene", "group"])
def test_register_sharded_real_oanet_two_processes(gpu, tmp_path, guard):
    import torch
    sys.path.insert(0, os.path.join(HERE, "helpers"))
    from dist_worker import case
    from lib import distributed as D
    world = 2
    env = dict(os.environ, WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    procs = [subprocess.Popen([sys.executable, WORKER, guard, str(tmp_path)], env=dict(env, RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(world)]
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace")[-3000:])
    assert all(p.returncode == 0 for p in procs), logs
    # one process over the whole batch, same guard / BatchNorm scope
    net, X = case(guard, gpu)
    with torch.no_grad():
        ref = D.register_pairs_sharded(net, {"xs": X}, 1, 0, guard=guard).cpu().numpy()
        net.guard_group = net.bn_group = D.GROUP if guard == "group" else 0
        plain = net({"xs": X})
    assert ref.shape == (70, D.REC)
    for r in range(world):
        rec = np.load(os.path.join(str(tmp_path), "rec_%d.npy" % r))
        np.testing.assert_array_equal(rec[:, 0], np.arange(70))
        # (pairs 32-63 are degenerate for the Procrustes: whatever it returns there must match too)
        assert np.array_equal(rec, ref, equal_nan=True), (r, np.nanmax(np.abs(rec - ref)))
    # the guard really fired, for a reason that lives on rank 0 only: pairs 32-63 have no positive logit in
    # block 0; every pair in its scope then carries + 1/N (scene: all 70, rank 1's 64-69 included; group: 32-63)
    lg = plain["logits"][0].cpu().numpy()
    sc = plain["scores"][0].cpu().numpy()
    zero_rows = np.where((lg > 0).sum(1) == 0)[0]
    assert len(zero_rows) > 0 and zero_rows.min() >= 32 and zero_rows.max() < 64, zero_rows
    scope = np.arange(70) if guard == "scene" else np.arange(32, 64)
    assert np.all(sc[scope] >= np.float32(1.0 / 1000) * 0.999)
    if guard == "group":
        assert np.any(sc[:32] == 0) and np.any(sc[64:] == 0)
