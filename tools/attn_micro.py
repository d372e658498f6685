"""Micro-benchmark of the fused diff_pool / diff_unpool kernels (csrc/oan_attn.hip) at the scene
shape (435 pairs x 5000 points, 128 channels, 500 clusters), timed with HIP events.
usage: python tools/attn_micro.py [--iters N] [--only pool|unpool]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d_multiview_reg_amd"))
import torch  # noqa: E402
from lib import _native as NV  # noqa: E402

P, N, C, K = 435, 5000, 128, 500
PEAK = 16 * 157.3 / 6   # split-bf16 fp32-equivalent TF/s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--clusters", type=int, default=K)
    ap.add_argument("--points", type=int, default=N)
    ap.add_argument("--math", type=int, default=-1, help="1 split-fp16, 0 split-bf16, -1 both (+ max difference)")
    ap.add_argument("--trace", action="store_true", help="library built with -DATTN_TRACE=1 (MVR_LIB): phase shares")
    a = ap.parse_args()
    run(a, a.clusters, a.points)


def run(a, K, N):
    d = torch.device("cuda")
    g = torch.Generator(device=d).manual_seed(0)
    x = torch.randn(P, C, N, device=d, generator=g)
    sc = torch.rand(P, C, device=d, generator=g) + 0.5
    sh = torch.rand(P, C, device=d, generator=g) - 0.5
    W = torch.randn(K, C, device=d, generator=g) * 0.1
    b = torch.randn(K, device=d, generator=g) * 0.1
    xd = torch.randn(P, C, K, device=d, generator=g)
    out_d = torch.empty(P, C, K, device=d)
    out_u = torch.empty(P, C, N, device=d)
    st_d = torch.empty(P, (K + 127) // 128, C, 2, device=d)
    st_u = torch.empty(P, (N + 127) // 128, C, 2, device=d)
    L = NV.lib()
    ws = max(L.mvr_oan_diff_unpool_workspace_bytes(P, C, K), L.mvr_oan_diff_pool_workspace_bytes(P, C, K))
    wbuf = torch.empty(ws, dtype=torch.uint8, device=d)
    s = NV.stream()

    def pool():
        assert L.mvr_oan_diff_pool_ws(NV.ptr(x), C * N, N, NV.ptr(sc), NV.ptr(sh), C, NV.ptr(W), NV.ptr(b), P, C, N,
                                      K, NV.ptr(out_d), C * K, K, NV.ptr(st_d), C, 0, NV.ptr(wbuf), ws, s) == 0

    def unpool():
        assert L.mvr_oan_diff_unpool(NV.ptr(x), C * N, N, NV.ptr(sc), NV.ptr(sh), C, NV.ptr(W), NV.ptr(b), NV.ptr(xd),
                                     C * K, K, P, C, N, K, NV.ptr(out_u), C * N, N, NV.ptr(st_u), C, 0, NV.ptr(wbuf),
                                     ws, s) == 0

    flops = 4.0 * C * K * N * P
    print("P=%d N=%d clusters=%d" % (P, N, K))
    maths = [a.math] if a.math >= 0 else [0, 1]
    for name, fn, o in (("pool", pool, out_d), ("unpool", unpool, out_u)):
        if a.only and a.only != name:
            continue
        res = {}
        for mth in maths:
            L.mvr_set_math(mth)
            fn()
            torch.cuda.synchronize()
            res[mth] = o.clone()
            time_it(a, name + "/h%d" % mth, fn, flops)
            if a.trace:
                import ctypes
                L.mvr_attn_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
                buf = (ctypes.c_ulonglong * 16)()
                L.mvr_attn_trace(buf, 1)
                fn()
                torch.cuda.synchronize()
                L.mvr_attn_trace(buf, 1)
                base = 0 if name == "pool" else 8
                names = (["prologue", "S mfma (+V split)", "softmax+P split", "O mfma (+K split)", "stage-end wait",
                          "split merge", "epilogue", "tail"] if name == "pool" else
                         ["prologue", "S mfma", "softmax+split", "x_down wait+barrier", "O mfma", "barrier+issue",
                          "epilogue", "tail"])
                tot = sum(buf[base + q] for q in range(8))
                print("   phase shares: " + ", ".join("%s %.1f%%" % (names[q], 100.0 * buf[base + q] / max(tot, 1))
                                                    for q in range(8)), flush=True)
        if len(res) == 2:
            d = (res[0] - res[1]).abs().max().item()
            print("%-7s max |h1 - h0| %.3e (max |out| %.3e)" % (name, d, res[0].abs().max().item()), flush=True)
        L.mvr_set_math(1)


def time_it(a, name, fn, flops):
    if True:
        for _ in range(2):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        print("%-7s %.3f ms  %.1f TF/s  (%.2f of split peak)" % (name, ms, flops / ms / 1e9, flops / ms / 1e9 / PEAK),
              flush=True)


if __name__ == "__main__":
    main()
