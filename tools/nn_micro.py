"""Micro-benchmark of the fused feature-NN kernel (csrc/feat_nn.hip) at the scene shape:
30 fragments x 5000 unit-norm 32-d descriptors, all 435 pairs, soft mode, tau = 0.3.
usage: python tools/nn_micro.py [--iters N] [--mode 0|1]"""
import argparse
import itertools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d_multiview_reg_amd"))
import torch  # noqa: E402
from lib import _native as NV  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--frags", type=int, default=30)
    ap.add_argument("--fast", type=int, default=1)
    ap.add_argument("--no-ws", action="store_true")
    a = ap.parse_args()
    d = torch.device("cuda")
    B, N, C = a.frags, 5000, 32
    g = torch.Generator(device=d).manual_seed(0)
    F = torch.randn(B, N, C, device=d, generator=g)
    F = F / F.norm(dim=-1, keepdim=True)
    X = torch.rand(B, N, 3, device=d, generator=g)
    pairs = torch.tensor(list(itertools.combinations(range(B), 2)), dtype=torch.int64, device=d)
    P = pairs.shape[0]
    out = torch.empty(P, N, 6, device=d)
    L = NV.lib()
    L.mvr_set_math(1 if a.fast == 2 else 0)
    L.mvr_debug_force(0, 1 if a.fast == 0 else 0)   # feat_nn_online

    nb = L.mvr_feat_nn_workspace_bytes(B, N)
    ws = torch.empty(nb, dtype=torch.uint8, device=d)

    def go():   # the pipeline's form: targets pre-split into the workspace (mvr_feat_nn_ws); --no-ws: mvr_feat_nn
        args = (NV.ptr(F), N * C, NV.ptr(F), N * C, NV.ptr(X), N * 3, NV.ptr(X), N * 3, NV.ptr(pairs), P, N, N,
                C, 1.0 / 0.09, a.mode, NV.ptr(out), N * 6, 6, None)
        rc = L.mvr_feat_nn(*args, NV.stream()) if a.no_ws else L.mvr_feat_nn_ws(*args, B, NV.ptr(ws), nb, NV.stream())
        assert rc == 0
    for _ in range(2):
        go()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(a.iters):
        go()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    el = float(P) * N * N
    print("feat_nn mode %d fast %d: %.3f ms  %.1f G elements/s  %.1f TF/s (distance GEMM, fp32-equivalent)"
          % (a.mode, a.fast, ms, el / ms / 1e6, 2 * el * C / ms / 1e9), flush=True)
