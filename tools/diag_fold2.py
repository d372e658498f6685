"""Folded vs materialised conv1 (mvr_set_oan_fused 5 vs 1) against the fp32 and fp64 numpy oracles over
several seeds: max |dR| per path (diagnostic for the sensitivity of random OANet weights)."""
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
for npts, seed in ((517, 23), (517, 5), (1234, 23), (2000, 31), (800, 3), (3000, 12)):
    xs, _, _ = synth_correspondences(5, npts, seed=seed)
    net = _oanet(128, 500, 9, gpu, which="full")
    st = synth_state(_shapes("full"), seed=9)
    o32 = oanet_forward(st, xs)
    o64 = oanet_forward(st, xs, dtype=np.float64)
    res = {}
    for f in (5, 1):
        L.mvr_set_oan_fused(f)
        with torch.no_grad():
            res[f] = net({"xs": torch.from_numpy(xs).unsqueeze(1)})
    L.mvr_set_oan_fused(5)
    i = 1
    d = lambda a, b: np.abs(a - b).reshape(5, -1).max(1)
    print("N %d seed %d  o32-o64 %s" % (npts, seed, np.array2string(d(o32["rot_est"][i], o64["rot_est"][i]), precision=1)))
    for f in (5, 1):
        R = res[f]["rot_est"][i].cpu().numpy()
        print("   fused %d: vs o32 %s  vs o64 %s" % (f, np.array2string(d(R, o32["rot_est"][i]), precision=1),
                                                  np.array2string(d(R, o64["rot_est"][i]), precision=1)), flush=True)
