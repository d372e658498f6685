"""Repeated forwards of one OANet case in one process (the flag-slot / epoch counters of the guarded split-fp16
launches advance by ~40 per forward, so 40 forwards cover every slot offset): any output that differs bitwise
from the first forward names a history-dependent path.  usage: python tools/diag_repeat.py [--reps 40]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "3d_multiview_reg_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    a = ap.parse_args()
    from test_gpu_oanet import _oanet
    from synth import synth_correspondences
    from lib import _native as NV
    gpu = torch.device("cuda:0")
    L = NV.lib()
    for npts, train, fused in ((1200, True, 5), (1200, True, 1), (2000, False, 5)):
        xs, _, _ = synth_correspondences(5, npts, seed=23)
        net = _oanet(128, 500, 9, gpu, train=train, which="full")
        prev = L.mvr_set_oan_fused(fused)
        outs = []
        for _ in range(a.reps):
            with torch.no_grad():
                o = net({"xs": torch.from_numpy(xs).unsqueeze(1)})
            outs.append(np.concatenate([o["logits"][i].cpu().numpy().ravel() for i in range(2)]))
        L.mvr_set_oan_fused(prev)
        bad = [i for i, x in enumerate(outs) if not np.array_equal(x, outs[0])]
        dmax = max((float(np.abs(outs[i] - outs[0]).max()) for i in bad), default=0.0)
        print("npts %d train %d fused %d: %d of %d forwards differ from the first (max %.3g) %s"
              % (npts, train, fused, len(bad), a.reps, dmax, bad[:10]), flush=True)


if __name__ == "__main__":
    main()
