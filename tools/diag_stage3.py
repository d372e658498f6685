"""Repeated OANet forwards with stage hashes, plus a dump of one stage's statistics partials
(mvr_debug_stage_dump): which (pair, tile, channel) partials differ between runs.
usage: python tools/diag_stage3.py [runs] [stage]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "3d_multiview_reg_amd"), ROOT, os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import torch  # noqa: E402
import bench  # noqa: E402
from lib import _native as NV  # noqa: E402


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    stage = int(sys.argv[2]) if len(sys.argv) > 2 else 14
    dev = torch.device("cuda")
    wl = bench.PrecomputedWorkload(dev, 0, 435, 5000)
    L = NV.lib()
    P, T, C = 435, 40, 128
    hs, dumps = [], []
    with torch.no_grad():
        for _ in range(runs):
            buf = torch.zeros(256, dtype=torch.int64, device=dev)
            dmp = torch.full((P, T, C, 2), float("nan"), device=dev)
            L.mvr_debug_stage_dump(stage, NV.ptr(dmp), dmp.numel() * 4)
            L.mvr_debug_stage_hash(NV.ptr(buf), 256)
            wl.step()
            L.mvr_debug_stage_hash(None, 0)
            hs.append(buf)
            dumps.append(dmp)
    torch.cuda.synchronize()
    h0 = hs[1].tolist()
    n = max(i for i, v in enumerate(h0) if v) + 1
    firsts = [next((i for i in range(n) if h.tolist()[i] != h0[i]), None) for h in hs[1:]]
    print("first differing stage per run (vs run 1):", firsts, flush=True)
    d0 = dumps[1]
    for r in range(2, runs):
        bad = (dumps[r] != d0) & ~(torch.isnan(dumps[r]) & torch.isnan(d0))
        if bad.any():
            idx = bad.nonzero()
            pt = sorted({(int(a), int(b)) for a, b, _, _ in idx.tolist()})
            chans = sorted({int(c) for _, _, c, _ in idx.tolist()})
            print("run %d: %d partials differ; (pair, tile): %s%s; channels %s" % (
                r, int(bad.sum()), pt[:12], " ..." if len(pt) > 12 else "", chans[:40]), flush=True)
            a, b, c, k = idx[0].tolist()
            print("   e.g. [%d,%d,%d,%d]: %r vs %r" % (a, b, c, k, dumps[r][a, b, c].tolist(), d0[a, b, c].tolist()))


if __name__ == "__main__":
    main()
