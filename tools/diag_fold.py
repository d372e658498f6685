import sys, numpy as np, torch
sys.path[:0] = ["/root/repo/3d_multiview_reg_amd", "/root/repo", "/root/repo/tests", "/root/repo/tests/golden"]
from lib import _native as NV
from test_gpu_oanet import _oanet
from synth import synth_correspondences
from oracle.oanet import oanet_forward
gpu = torch.device("cuda")
for npts in (33, 65, 517):
    xs, _, _ = synth_correspondences(5, npts, seed=23)
    net = _oanet(128, 500, 9, gpu, which="full")
    st = {k: v.detach().cpu().numpy() for k, v in net.state_dict().items()}
    ref = oanet_forward(st, xs)
    L = NV.lib()
    res = {}
    for f in (5, 1, 0):
        L.mvr_set_oan_fused(f)
        with torch.no_grad():
            res[f] = net({"xs": torch.from_numpy(xs).unsqueeze(1)})
    L.mvr_set_oan_fused(5)
    for f in (5, 1, 0):
        for i in range(2):
            dl = np.abs(res[f]["logits"][i].cpu().numpy() - ref["logits"][i]).max()
            dR = np.abs(res[f]["rot_est"][i].cpu().numpy() - ref["rot_est"][i]).max()
            print("N %d fused %d block %d: |dlogit| %.2e |dR| %.2e vs fp64 oracle" % (npts, f, i, dl, dR), flush=True)
