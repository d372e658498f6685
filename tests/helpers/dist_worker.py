"""One rank of the multi-process sharded-registration GPU test (tests/test_gpu_distributed.py): the real OANet
(RegBlock size) through lib.distributed.register_pairs_sharded on cuda:0, gloo process group (several ranks share
the box's one GPU; gloo moves host tensors, so lib.distributed stages the collectives through host memory).
Writes this rank's gathered records to <out>/rec_<rank>.npy.

usage: RANK=r WORLD_SIZE=w MASTER_ADDR=127.0.0.1 MASTER_PORT=p python tests/helpers/dist_worker.py <guard> <out>"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "3d_multiview_reg_amd"), ROOT, os.path.join(ROOT, "tests", "golden"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def case(guard, dev):
    """the shared input: 70 pairs x 1000 correspondences; pairs 32-63 are all-zero correspondences (every
    correspondence of such a pair is the same input, so the pair has a single logit value), and block 0's output
    bias is shifted — from a probe forward of this very batch, in this mode — so that this value is negative while
    every other pair keeps a positive logit.  The zero-row guard then fires for pairs 32-63 only, all on rank 0 at
    world 2 (rank 0 holds pairs 0-63, rank 1 pairs 64-69).  guard 'scene': eval mode (the guard over the whole
    batch); 'group': train mode (BatchNorm statistics and guard per 32-pair group, the benchmark's loader batches)."""
    from lib.filtering.oanet import OANet
    from lib import distributed as D
    from synth import synth_state, synth_correspondences
    cfg = {"misc": {"net_depth": 12, "clusters": 500, "iter_num": 1, "net_channel": 128, "use_gpu": True,
                    "normalize_weights": True}, "data": {"use_mutuals": 0}}
    net = OANet(cfg)
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    st = synth_state(shapes, seed=7)
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    net = net.to(dev).train(guard == "group")
    xs, _, _ = synth_correspondences(70, 1000, seed=29)
    xs[32:64] = 0.0
    X = torch.from_numpy(xs).unsqueeze(1).to(dev)
    net.guard_group = net.bn_group = D.GROUP if guard == "group" else 0
    with torch.no_grad():
        lg = net({"xs": X})["logits"][0].float().cpu().numpy()
    zmax = lg[32:64].max()
    omin = np.concatenate([lg[:32], lg[64:]]).max(1).min()
    assert zmax < omin, ("probe: the all-zero pairs' logit is not below every other pair's maximum", zmax, omin)
    with torch.no_grad():
        net.reg_init.output.bias -= float(zmax + omin) / 2
    net.guard_group = net.bn_group = 0
    return net, X


def main():
    guard, out = sys.argv[1], sys.argv[2]
    import torch.distributed as dist
    from lib import distributed as D
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        net, X = case(guard, dev)
        with torch.no_grad():
            rec = D.register_pairs_sharded(net, {"xs": X}, world, rank, guard=guard)
        torch.cuda.synchronize()
        np.save(os.path.join(out, "rec_%d.npy" % rank), rec.cpu().numpy())
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
