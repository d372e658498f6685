"""Numerics diagnostic: GPU OANet vs the numpy oracle in fp32 and fp64 (ragged N)."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden"), ROOT,
                os.path.join(ROOT, "3d_multiview_reg_amd")]
import torch  # noqa: E402
from synth import synth_correspondences, synth_state  # noqa: E402
from oracle.oanet import oanet_forward  # noqa: E402
import test_gpu_oanet as T  # noqa: E402

for (P, N, seed) in [(5, 1234, 77), (4, 2000, 5)]:
    xs, _, _ = synth_correspondences(P, N, seed=seed)
    net = T._oanet(128, 500, 7, torch.device("cuda"), which="full")
    with torch.no_grad():
        out = net({"xs": torch.from_numpy(xs).unsqueeze(1)})
    st = synth_state(T._shapes("full"), seed=7)
    o32 = oanet_forward(st, xs)
    o64 = oanet_forward(st, xs, dtype=np.float64)
    for i in range(2):
        lg = out["logits"][i].cpu().numpy()
        R = out["rot_est"][i].cpu().numpy()
        print("P=%d N=%d blk%d  logit gpu-o32 %.2e gpu-o64 %.2e o32-o64 %.2e | R gpu-o32 %.2e gpu-o64 %.2e o32-o64 %.2e"
              % (P, N, i, np.abs(lg - o32["logits"][i]).max(), np.abs(lg - o64["logits"][i]).max(),
                 np.abs(o32["logits"][i] - o64["logits"][i]).max(), np.abs(R - o32["rot_est"][i]).max(),
                 np.abs(R - o64["rot_est"][i]).max(), np.abs(o32["rot_est"][i] - o64["rot_est"][i]).max()),
              flush=True)
