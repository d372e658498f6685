"""OANet forward alone, repeated on the same input with per-stage hashes (mvr_debug_stage_hash): which
stages vary run to run.  usage: [MVR_LIB=...] python tools/diag_stage2.py [runs]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "3d_multiview_reg_amd"), ROOT, os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from lib import _native as NV  # noqa: E402


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    dev = torch.device("cuda")
    wl = bench.PrecomputedWorkload(dev, 0, 435, 5000)
    L = NV.lib()
    hs = []
    with torch.no_grad():
        for _ in range(runs):
            buf = torch.zeros(256, dtype=torch.int64, device=dev)
            L.mvr_debug_stage_hash(NV.ptr(buf), 256)
            wl.step()
            L.mvr_debug_stage_hash(None, 0)
            hs.append(buf)
    torch.cuda.synchronize()
    h0 = hs[1].tolist()   # run 0 hashes leftovers of never-written halves (st11 rows C..2C) differently
    n = max(i for i, v in enumerate(h0) if v) + 1
    firsts = [next((i for i in range(n) if h.tolist()[i] != h0[i]), None) for h in hs[1:]]
    print(os.environ.get("MVR_LIB", "default"), "stages", n, "first differing stage per run (vs run 1)", firsts,
          flush=True)
    classes = {}
    for r, h in enumerate(hs):
        classes.setdefault(tuple(h.tolist()[:n]), []).append(r)
    print("distinct stage-hash vectors: %d; runs per class: %s" % (len(classes), list(classes.values())), flush=True)


if __name__ == "__main__":
    main()
