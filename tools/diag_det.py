"""Run-to-run determinism of the OANet forward (same inputs twice, bitwise compare), eval and train BN."""
import sys
import numpy as np
import torch
sys.path[:0] = ["/root/repo/3d_multiview_reg_amd", "/root/repo", "/root/repo/tests", "/root/repo/tests/golden"]
from lib import _native as NV
from test_gpu_oanet import _oanet
from synth import synth_correspondences
gpu = torch.device("cuda")
L = NV.lib()
for train in (False, True):
    for f in (5, 1):
        xs, _, _ = synth_correspondences(5, 1200, seed=23)
        net = _oanet(128, 500, 9, gpu, train=train, which="full")
        L.mvr_set_oan_fused(f)
        outs = []
        for rep in range(3):
            with torch.no_grad():
                o = net({"xs": torch.from_numpy(xs).unsqueeze(1)})
            outs.append({k: [v.cpu().numpy() for v in o[k]] for k in ("logits", "rot_est")})
        for rep in (1, 2):
            dl = max(np.abs(outs[0]["logits"][i] - outs[rep]["logits"][i]).max() for i in range(2))
            dr = max(np.abs(outs[0]["rot_est"][i] - outs[rep]["rot_est"][i]).max() for i in range(2))
            print("train %d fused %d rep %d: max |dlogit| %.3e |dR| %.3e" % (train, f, rep, dl, dr), flush=True)
L.mvr_set_oan_fused(5)
