"""Micro-benchmark of the fused PointCN kernel (csrc/pointcn.hip) and of the two GEMMs it replaces,
at the scene shape (435 pairs x 5000 points x 128 channels), timed with HIP events.
usage: python tools/pcn_micro.py [--iters N]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d_multiview_reg_amd"))
import torch  # noqa: E402
from lib import _native as NV  # noqa: E402

P, N, C = 435, 5000, 128


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--points", type=int, default=N)
    a = ap.parse_args()
    n = a.points
    d = torch.device("cuda")
    g = torch.Generator(device=d).manual_seed(0)
    x = torch.randn(P, C, n, device=d, generator=g)
    y = torch.empty_like(x)
    f = [torch.rand(P, C, device=d, generator=g) + 0.5 for _ in range(4)]
    W = [torch.randn(C, C, device=d, generator=g) * 0.1 for _ in range(2)]
    b = [torch.randn(C, device=d, generator=g) * 0.1 for _ in range(2)]
    st = torch.empty(P, (n + 31) // 32, C, 2, device=d)
    L = NV.lib()
    s = NV.stream()

    def pcn():
        assert L.mvr_pointcn_fused(NV.ptr(x), C * n, n, NV.ptr(y), C * n, n, NV.ptr(f[0]), NV.ptr(f[1]), NV.ptr(f[2]),
                                   NV.ptr(f[3]), NV.ptr(W[0]), NV.ptr(b[0]), NV.ptr(W[1]), NV.ptr(b[1]), P, C, n,
                                   NV.ptr(st), C, 0, s) == 0
    for _ in range(2):
        pcn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(a.iters):
        pcn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    byt = 2.0 * 4 * C * n * P
    print("pointcn %.3f ms  %.0f GB/s  %.1f TF/s" % (ms, byt / ms / 1e6, 4.0 * C * C * n * P / ms / 1e9), flush=True)


if __name__ == "__main__":
    main()
