"""Block-0 logits of the folded (5) and materialised (1) conv1 paths against the fp64 numpy oracle
(the well-conditioned part of the network), eval and train-mode BN, several seeds."""
import sys
import numpy as np
import torch
sys.path[:0] = ["/root/repo/3d_multiview_reg_amd", "/root/repo", "/root/repo/tests", "/root/repo/tests/golden"]
from lib import _native as NV
from test_gpu_oanet import _oanet, _shapes
from synth import synth_correspondences, synth_state
from oracle.oanet import oanet_forward
gpu = torch.device("cuda")
L = NV.lib()
for train in (False, True):
    for npts, seed in ((517, 23), (1200, 23), (2000, 31), (3000, 12)):
        xs, _, _ = synth_correspondences(5, npts, seed=seed)
        net = _oanet(128, 500, 9, gpu, train=train, which="full")
        st = synth_state(_shapes("full"), seed=9)
        o32 = oanet_forward(st, xs, train=train)
        o64 = oanet_forward(st, xs, train=train, dtype=np.float64)
        res = {}
        for f in (5, 1):
            L.mvr_set_oan_fused(f)
            with torch.no_grad():
                res[f] = net({"xs": torch.from_numpy(xs).unsqueeze(1)})
        L.mvr_set_oan_fused(5)
        line = "train %d N %d seed %d  o32: %.2e" % (train, npts, seed, np.abs(o32["logits"][0] - o64["logits"][0]).max())
        for f in (5, 1):
            for i in range(2):
                line += "  f%d b%d %.2e" % (f, i, np.abs(res[f]["logits"][i].cpu().numpy() - o64["logits"][i]).max())
        print(line, flush=True)
