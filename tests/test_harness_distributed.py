"""The evaluation harness sharded over ranks (scripts/benchmark_pairwise_registration.py
under torchrun) on CPU with gloo: the file list of the whole evaluation split into contiguous blocks of whole
loader batches (lib/data.py make_pairwise_eval_data_loader), the per-pair records all-gathered, traj.txt and the
report written by rank 0.  The per-batch GPU work is replaced by a deterministic CPU stand-in (helpers/
harness_worker.py stub_batch_records, a function of the batch, its GLOBAL batch index and the pair index), so the
test pins the host logic: the trajectories and the summary of 2 and 3 ranks are byte-identical to one process —
batches that straddle a scene boundary, a rank with an empty block, the mutuals mode (batch size 1)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import GOLDEN

HERE = os.path.dirname(os.path.abspath(__file__))
HELPERS = os.path.join(HERE, "helpers")
if HELPERS not in sys.path:
    sys.path.insert(0, HELPERS)
WORKER = os.path.join(HELPERS, "harness_worker.py")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run_ranks(world, out, cwd, argv, stub, extra_env=None, timeout=300):
    """world processes of helpers/harness_worker.py (torchrun's environment, gloo); their summaries"""
    env = dict(os.environ, WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               **(extra_env or {}))
    cmd = [sys.executable, WORKER, out, cwd] + (["stub"] if stub else []) + ["--"] + argv
    procs = [subprocess.Popen(cmd, env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT) for r in range(world)]
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace")[-3000:])
    assert all(p.returncode == 0 for p in procs), logs
    return [json.load(open(os.path.join(out, "summary_%d.json" % r))) for r in range(world)]


@pytest.mark.parametrize("world,mutuals", [(2, False), (3, False), (2, True)])
def test_harness_sharded_equals_one_process(tmp_path, world, mutuals):
    from eval_layout import write_eval, read_results
    argv_for = lambda root: ["--source_path", root, "--method", "RANSAC", "--batch_size", "32",  # noqa: E731
                             "--num_workers", "0", "--dist_backend", "gloo"] + (["--mutuals"] if mutuals else [])
    one, many = str(tmp_path / "one"), str(tmp_path / "many")
    for root in (one, many):
        write_eval(root)
    # 51 pairs in batches of 32: world 3 leaves rank 2 an empty block; with --mutuals (batch 1) 51 single-pair
    # batches over the ranks
    s1 = run_ranks(1, one, GOLDEN, argv_for(one), stub=True)[0]
    sN = run_ranks(world, many, GOLDEN, argv_for(many), stub=True)
    r1, rN = read_results(one, "3d_match", "RANSAC", mutuals), read_results(many, "3d_match", "RANSAC", mutuals)
    assert sorted(r1) == ["kitchen", "sun3d-hotel_uc-scan3"]
    assert r1 == rN                                                  # byte-identical trajectories
    n_written = len(r1["kitchen"].splitlines()) // 5                  # pairs past the (stub) overlap gate
    assert 0 < n_written < 36
    for s in sN:                                                     # every rank returns rank 0's summary
        assert json.dumps(s, sort_keys=True) == json.dumps(s1, sort_keys=True)


def test_sharded_loader_blocks_are_whole_batches(tmp_path):
    """lib.data.make_pairwise_eval_data_loader(world, rank): contiguous blocks of whole batches, global indices,
    the whole evaluation's scene_info on every rank"""
    import argparse
    from eval_layout import write_eval
    from lib.data import make_pairwise_eval_data_loader
    write_eval(str(tmp_path))
    args = argparse.Namespace(source_path=os.path.join(str(tmp_path), "3d_match"), method="RANSAC", mutuals=False,
                              overwrite=False, only_gt_overlaping=False, batch_size=32)
    full, info = make_pairwise_eval_data_loader(args, num_workers=0)
    idx_full = [int(i) for b in full for i in b["idx"]]
    assert idx_full == list(range(51)) and info["nr_examples"] == 51 and full.pair_block == (0, 51)
    for world in (2, 3, 8):
        got = []
        for r in range(world):
            ld, inf = make_pairwise_eval_data_loader(args, num_workers=0, world=world, rank=r)
            assert inf == info
            s, e = ld.pair_block
            assert s % 32 == 0 or s == e
            batches = [[int(i) for i in b["idx"]] for b in ld]
            assert all(len(b) == 32 for b in batches[:-1])
            got += [i for b in batches for i in b]
        assert got == idx_full
