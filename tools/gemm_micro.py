"""Micro-benchmark of the fused GEMM kernels at OANet shapes (timing with HIP events).
usage: python tools/gemm_micro.py [--iters N] [--only NAME]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d_multiview_reg_amd"))
import torch  # noqa: E402
from lib import _native as NV  # noqa: E402

P, N, C, K = 435, 5000, 128, 500
CASES = {
    # name: (M, N, K, pro, bkc, bias, stats, res)
    "conv_plain": (C, N, C, 0, 0, 0, 0, 0),
    "conv_pro_stats": (C, N, C, 2, 0, 1, 1, 0),
    "conv_res": (C, N, C, 2, 0, 1, 1, 1),
    "conv256_pro_stats": (C, N, 2 * C, 2, 0, 1, 1, 0),   # PointCN(2C -> C) conv3
    "conv256_plain": (C, N, 2 * C, 0, 0, 1, 0, 0),       # PointCN(2C -> C) shortcut
    "embed_rowsmx": (K, N, C, 2, 0, 1, 2, 0),
    "pool": (C, K, N, 3, 1, 0, 1, 0),
    "unpool": (C, N, K, 3, 0, 0, 1, 0),
    "oaf_conv2": (C, K, K, 1, 1, 2, 1, 1),    # OAFilter conv2 (oanet.hip oafilter): W2 shared, bias per n, residual
    "oaf_conv2_so": (C, K, K, 1, 1, 2, 1, 1),  # the same on the split-once kernel (mvr_oaf_conv2_f32)
    "conv_oaf1": (C, K, C, 2, 0, 1, 4, 0),    # OAFilter conv1 over the clusters: IN/BN/ReLU prologue, column stats
}


TRACE = False
PTRACE = False
PGRID = 1


def run(name, iters, math, pconv=1):
    M, Nn, Kk, pro, bkc, bias, stats, res = CASES[name]
    d = torch.device("cuda")
    A = torch.randn(M, Kk, device=d) * 0.1 if name.startswith(("conv", "embed")) else torch.randn(P, M, Kk, device=d)
    sAb = 0 if A.dim() == 2 else M * Kk
    Nl = (Nn + 31) // 32 * 32   # 128-byte rows, as the OANet activations (csrc/oanet.hip plan)
    Bt = torch.randn(P, Nn, Kk, device=d) if bkc else torch.randn(P, Kk, Nl, device=d)
    sBb = (Nn * Kk if bkc else Kk * Nl)
    if name.startswith("oaf"):   # the weight operand is shared by all pairs
        Bt, sBb = torch.randn(Nn, Kk, device=d) * 0.05, 0
    Cout = torch.empty(P, M, Nl, device=d)
    R = torch.randn(P, M, Nl, device=d) if res else None
    bvec = torch.randn(M if bias == 1 else Nn, device=d) if bias else None
    kt = (Kk + 127) // 128
    if pro in (1, 2):
        sc, sh, sPb, pld = torch.rand(P, Kk, device=d) + 0.5, torch.rand(P, Kk, device=d), Kk, 0
    elif pro == 3:
        sc, sh, sPb, pld = torch.rand(P, kt, Nn, device=d), None, kt * Nn, Nn
    else:
        sc = sh = None
        sPb = pld = 0
    nt = (Nn + 127) // 128
    mt = (M + 127) // 128
    st = torch.empty(P, max(nt, mt), max(M, Nn), 2, device=d) if stats else None
    st_ld = M if stats in (1, 2) else Nn
    L = NV.lib()
    L.mvr_debug_force(1, 0 if pconv else 1)   # generic_gemm
    so = name.startswith("oaf_conv2_so")
    img = torch.empty(int(L.mvr_oaf_conv2_image_bytes(Nn, Kk)) // 4 + 4, device=d) if so else None

    def go():
        if img is not None:
            rc = L.mvr_oaf_conv2_f32(M, Nn, Kk, P, NV.ptr(A), sAb, Kk, NV.ptr(Bt), Kk, NV.ptr(Cout), M * Nl, Nl,
                                     NV.ptr(R), M * Nl, NV.ptr(bvec), NV.ptr(sc), NV.ptr(sh), sPb, NV.ptr(st), st_ld,
                                     NV.ptr(img), img.numel() * 4, NV.stream())
            assert rc == 0
            return
        rc = L.mvr_gemm_f32(M, Nn, Kk, P, NV.ptr(A), sAb, Kk, NV.ptr(Bt), sBb, Kk if bkc else Nl, bkc,
                            NV.ptr(Cout), M * Nl, Nl, NV.ptr(R), M * Nl, NV.ptr(bvec), bias, NV.ptr(sc),
                            NV.ptr(sh), sPb, pld, pro, NV.ptr(st), st_ld, 0, stats, math, NV.ptr(NV.flag_word()), NV.stream())
        assert rc == 0
    for _ in range(2):
        go()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        go()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    fl = 2.0 * M * Nn * Kk * P
    by = 4.0 * P * (Kk * Nn + M * Nn * (2 if res else 1))
    print("P%-4d %-16s m%d%s %8.3f ms  %7.1f TF/s  %7.0f GB/s" % (P, name, math, " pconv" if pconv and M == C and Kk in (C, 2 * C) else "",
                                                          ms, fl / ms / 1e9, by / ms / 1e6), flush=True)
    if PTRACE:
        import ctypes
        buf = (ctypes.c_ulonglong * 8)()
        L.mvr_pconv_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.mvr_pconv_trace(buf, 1)
        go()
        torch.cuda.synchronize()
        L.mvr_pconv_trace(buf, 1)
        tot = sum(buf)
        names = ["mfma+split", "epilogue", "bookkeeping", "step barrier", "prologue", "tail", "-", "-"]
        print("   pconv phase shares (wave-cycles, one launch): " +
              ", ".join("%s %.1f%%" % (names[q], 100.0 * buf[q] / max(tot, 1)) for q in range(6)), flush=True)
    if TRACE:
        import ctypes
        buf = (ctypes.c_ulonglong * 8)()
        L.mvr_gemm_trace(buf, 1)
        go()
        torch.cuda.synchronize()
        L.mvr_gemm_trace(buf, 1)
        tot = sum(buf)
        names = ["stage-wait+barrier", "ktail+lds-reads", "barrier+issue", "transform+split+mfma",
                 "refill(late)/loop", "tile_of", "epilogue", "tail"]
        if name == "oaf_conv2_so":   # the split-once kernel's phases (gemm.hip oaf_conv2_kernel)
            names = ["barrier", "A-wait+DMA-issue", "k16 step 0 + split", "k16 step 1", "epilogue", "stage-end wait",
                     "-", "prologue/tail"]
        print("   phase shares (wave-cycles, one launch): " +
              ", ".join("%s %.1f%%" % (names[q], 100.0 * buf[q] / max(tot, 1)) for q in range(8)), flush=True)


def copy_bw(iters):
    d = torch.device("cuda")
    x = torch.randn(P, C, N, device=d)
    y = torch.empty_like(x)
    for _ in range(2):
        y.copy_(x)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        y.copy_(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    print("%-16s    %8.3f ms  %7.0f GB/s (read+write of the conv activation)" % ("copy", ms, 2 * x.numel() * 4 / ms / 1e6))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default=None)
    ap.add_argument("--math", default="01")
    ap.add_argument("--trace", action="store_true", help="library built with -DGEMM_TRACE=1 (MVR_LIB)")
    ap.add_argument("--ptrace", action="store_true", help="library built with -DPCONV_TRACE=1 (MVR_LIB): point-conv phases")
    ap.add_argument("--pairs", type=int, default=P, help="pair batch (small batches stay in the Infinity Cache)")
    ap.add_argument("--pconv-grid", type=int, default=1, help="mvr_set_pconv_grid")
    a = ap.parse_args()
    P = a.pairs
    PGRID = a.pconv_grid
    TRACE = a.trace
    PTRACE = a.ptrace
    if TRACE:
        import ctypes
        NV.lib().mvr_gemm_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
    copy_bw(a.iters)
    for n in CASES:
        if a.only and n != a.only:
            continue
        for m in a.math:
            run(n, a.iters, int(m), 0)
            if m == "1" and n.startswith("conv"):
                run(n, a.iters, int(m), 1)
