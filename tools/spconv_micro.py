"""Micro-benchmark of the sparse 3^3 convolution (csrc/spconv.hip) on a real kernel map: the synthetic
3DMatch-scale scene (tests/golden/synth.py, 30 fragments, 0.025 m voxels), every FCGF level, both
split-bf16 arithmetic with pre-split weights, timed with HIP events.
usage: python tools/spconv_micro.py [--frags 30] [--iters 10] [--only s1:1:64:64]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "3d_multiview_reg_amd"), ROOT, os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import torch  # noqa: E402
from lib import _native as NV  # noqa: E402

# (kernel-map kind, stride, Cin, Cout) of the FCGF convs (lib/descriptor/fcgf.py forward)
CASES = [("s1", 1, 32, 32), ("down", 1, 32, 64), ("s1", 2, 64, 64), ("down", 2, 64, 128), ("s1", 4, 128, 128),
         ("down", 4, 128, 256), ("s1", 8, 256, 256), ("up", 4, 256, 128), ("up", 2, 256, 64), ("up", 1, 128, 64),
         ("s1", 1, 64, 64)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frags", type=int, default=30)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default=None)
    ap.add_argument("--order", default=None, help="run only this row order (e.g. mask+morton)")
    ap.add_argument("--xcd", type=int, default=0, help="(tile order selector removed in round 5: 0 only)")
    ap.add_argument("--trace", action="store_true", help="library built with -DSP_TRACE=1 (MVR_LIB): phase shares")
    a = ap.parse_args()
    from synth import synth_scene_fragments
    from lib.sparse import voxelize, CoordinateManager
    dev = torch.device("cuda")
    frags, _ = synth_scene_fragments(a.frags, seed=41)
    c, _, counts, _ = voxelize([torch.from_numpy(f).to(dev) for f in frags], 0.025, dev)
    cm = CoordinateManager(c, len(frags))
    L = NV.lib()
    g = torch.Generator(device=dev).manual_seed(0)
    for kind, s, cin, cout in CASES:
        tag = "%s:%d:%d:%d" % (kind, s, cin, cout)
        if a.only and tag != a.only:
            continue
        nbr = cm.kernel_map(kind, s)
        perm = cm.kernel_map_order(kind, s)
        Mout = nbr.shape[0]
        Min = cm.coords_at(s if kind != "up" else 2 * s).shape[0] if kind != "down" else cm.coords_at(s).shape[0]
        x = torch.randn(Min, cin, device=dev, generator=g)
        W = torch.randn(27, cin, cout, device=dev, generator=g) / (27 * cin) ** 0.5
        out = torch.empty(Mout, cout, device=dev)
        nb = L.mvr_spconv_wimage_bytes(27, cin, cout)
        wimg = torch.empty(nb, dtype=torch.uint8, device=dev)
        NV.check(L.mvr_spconv_wimage(NV.ptr(W), 27, cin, cout, NV.ptr(wimg), nb, NV.stream()), "wimage")
        bn = NV.BnP(None, None, None, None)
        act = (nbr >= 0).sum().item()
        out_c = cm.coords_at(2 * s if kind == "down" else s)
        step = 2 * s if kind == "down" else s
        mask = ((nbr >= 0).to(torch.int64) << torch.arange(27, device=dev)).sum(1)
        q = (out_c[:, 1:].to(torch.int64) // step) & 511
        mort = torch.zeros_like(mask)
        for b in range(9):
            for ax in range(3):
                mort |= ((q[:, ax] >> b) & 1) << (3 * b + 2 - ax)
        mort |= (out_c[:, 0].to(torch.int64) & 31) << 27
        orders = {"none": None,
                  "mask": torch.argsort(mask, stable=True).to(torch.int32),
                  "mask+morton": perm,
                  "morton": torch.argsort(mort, stable=True).to(torch.int32),
                  "frag+mask": torch.argsort(((out_c[:, 0].to(torch.int64) & 31) << 32) | mask, stable=True).to(torch.int32),
                  # spatial cells (16^3 / 32^3 voxels of the level: the Morton code's top bits) first, mask inside
                  "cell12+mask": torch.argsort(((mort >> 12) << 27) | mask, stable=True).to(torch.int32),
                  "cell15+mask": torch.argsort(((mort >> 15) << 27) | mask, stable=True).to(torch.int32)}
        res = {}
        for oname, pm in orders.items():
            if a.order and oname != a.order:
                continue
            for xcd in (0, 1):
                if a.xcd is not None and xcd != a.xcd:
                    continue

                def go():
                    NV.check(L.mvr_spconv(NV.ptr(x), cin, cin, NV.ptr(nbr), NV.ptr(pm), 27, Mout, NV.ptr(W), cout, None,
                                          bn, 1e-5, None, 0, 0, NV.ptr(out), cout, NV.ptr(wimg), None, NV.stream()),
                             "spconv")
                for _ in range(2):
                    go()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(a.iters):
                    go()
                e1.record()
                torch.cuda.synchronize()
                res["%s/x%d" % (oname, xcd)] = e0.elapsed_time(e1) / a.iters
                if a.trace:
                    import ctypes
                    buf = (ctypes.c_ulonglong * 8)()
                    L.mvr_spconv_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
                    L.mvr_spconv_trace(buf, 1)
                    go()
                    torch.cuda.synchronize()
                    L.mvr_spconv_trace(buf, 1)
                    tot = max(sum(buf), 1)
                    names = ["setup", "w-store(+wait)", "A split", "gather issue", "mfma", "barrier", "epilogue",
                             "prologue"]
                    print("   %s phase shares: %s" % (tag, ", ".join("%s %.1f%%" % (names[q], 100.0 * buf[q] / tot)
                                                                     for q in range(8))), flush=True)
        fl = 2.0 * act * cin * cout
        print("%-16s Mout %7d active/row %.1f  %s   (useful TF/s at best %.1f)" % (
            tag, Mout, act / Mout, "  ".join("%s %.3f" % kv for kv in res.items()), fl / min(res.values()) / 1e9),
            flush=True)


if __name__ == "__main__":
    main()
