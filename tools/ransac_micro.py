"""Timing of the batched GPU RANSAC (csrc/procrustes.hip mvr_ransac) at the benchmark's --refine / RANSAC
baseline shape: P pairs x 5000 correspondences x 2500 iterations (lib/utils.py:671-709), HIP events, plus
the numpy restatement (oracle/ransac.py) on one pair with fewer iterations, scaled.
usage: python tools/ransac_micro.py [--pairs 435] [--iters 2500]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "3d_multiview_reg_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from lib import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=435)
    ap.add_argument("--n", type=int, default=5000)
    ap.add_argument("--iters", type=int, default=2500)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    d = torch.device("cuda")
    g = torch.Generator(device=d).manual_seed(0)
    x1 = torch.rand(a.pairs, a.n, 3, device=d, dtype=torch.float64, generator=g) * 3
    x2 = x1 + 0.01 * torch.randn(a.pairs, a.n, 3, device=d, dtype=torch.float64, generator=g)
    x2[:, a.n // 5:] = torch.rand(a.pairs, a.n - a.n // 5, 3, device=d, dtype=torch.float64, generator=g) * 3
    cnt = torch.full((a.pairs,), a.n, dtype=torch.int32, device=d)
    T = torch.empty(a.pairs, 4, 4, dtype=torch.float64, device=d)
    fit, rmse = (torch.empty(a.pairs, dtype=torch.float64, device=d) for _ in range(2))
    best = torch.empty(a.pairs, dtype=torch.int32, device=d)
    L = N.lib()
    ws = torch.empty(L.mvr_ransac_workspace_bytes(a.pairs, a.iters), dtype=torch.uint8, device=d)

    def run():
        assert L.mvr_ransac(N.ptr(x1), N.ptr(x2), a.n * 3, N.ptr(cnt), a.pairs, 4, a.iters, 0.05, 1, N.ptr(T),
                            N.ptr(fit), N.ptr(rmse), N.ptr(best), None, N.ptr(ws), ws.numel(), N.stream()) == 0
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    flop = 27.0 * a.pairs * a.iters * a.n   # 12 mul + 15 add/sub per (hypothesis, correspondence), fp64
    print("ransac %d pairs x %d corr x %d iters: %.3f ms  %.1f pairs/s  %.1f TF/s fp64 (of 78.6 vector)"
          % (a.pairs, a.n, a.iters, ms, a.pairs / ms * 1e3, flop / ms / 1e9), flush=True)
    print("fitness mean %.3f (inlier fraction 0.2)" % fit.mean().item(), flush=True)
    from oracle import ransac as O
    h1, h2 = x1[0].cpu().numpy(), x2[0].cpu().numpy()
    it = 40
    t0 = time.time()
    O.ransac(h1, h2, seed=1, iters=it)
    dt = (time.time() - t0) * a.iters / it
    print("numpy restatement (1 thread, vectorised over correspondences): %.2f s per pair (%d iters scaled "
          "from %d) = %.3f pairs/s" % (dt, a.iters, it, 1.0 / dt), flush=True)


if __name__ == "__main__":
    main()
