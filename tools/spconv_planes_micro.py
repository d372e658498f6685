"""Sparse conv (csrc/spconv.hip) with fp32 gathers split in the kernel (PS = 0) against pre-split bf16 planes
(PS = 1, mvr_spconv_x in_planes), on the real kernel maps of the synthetic 3DMatch-scale scene: ms per launch
(HIP events), outputs compared bit for bit, and the producer side (out_planes) checked against torch's split.
usage: python tools/spconv_planes_micro.py [--frags 30] [--iters 10] [--only s1:1:32:32]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "3d_multiview_reg_amd"), ROOT, os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import torch  # noqa: E402
from lib import _native as NV  # noqa: E402

CASES = [("s1", 1, 32, 32), ("down", 1, 32, 64), ("s1", 2, 64, 64), ("down", 2, 64, 128), ("s1", 4, 128, 128),
         ("down", 4, 128, 256), ("s1", 8, 256, 256), ("up", 4, 256, 128), ("up", 2, 256, 64), ("up", 1, 128, 64),
         ("s1", 1, 64, 64)]


def planes(x):
    """[M, C] fp32 -> [M, 3, C] int16: the RNE bf16 split h, m, l (x - h and r - m exact)"""
    h = x.to(torch.bfloat16)
    r = x - h.float()
    m = r.to(torch.bfloat16)
    lo = (r - m.float()).to(torch.bfloat16)
    return torch.stack([h, m, lo], 1).view(torch.int16).contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frags", type=int, default=30)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    from synth import synth_scene_fragments
    from lib.sparse import voxelize, CoordinateManager
    dev = torch.device("cuda")
    frags, _ = synth_scene_fragments(a.frags, seed=41)
    c, _, counts, _ = voxelize([torch.from_numpy(f).to(dev) for f in frags], 0.025, dev)
    cm = CoordinateManager(c, len(frags))
    cm.prepare_orders()
    L = NV.lib()
    g = torch.Generator(device=dev).manual_seed(0)
    tot = {0: 0.0, 1: 0.0}
    for kind, s, cin, cout in CASES:
        tag = "%s:%d:%d:%d" % (kind, s, cin, cout)
        if a.only and tag != a.only:
            continue
        nbr = cm.kernel_map(kind, s)
        perm = cm.kernel_map_order(kind, s)
        Mout = nbr.shape[0]
        Min = cm.coords_at(2 * s if kind == "up" else s).shape[0]
        x = torch.relu(torch.randn(Min, cin, device=dev, generator=g))
        xp = planes(x)
        W = torch.randn(27, cin, cout, device=dev, generator=g) / (27 * cin) ** 0.5
        nb = L.mvr_spconv_wimage_bytes(27, cin, cout)
        wimg = torch.empty(nb, dtype=torch.uint8, device=dev)
        NV.check(L.mvr_spconv_wimage(NV.ptr(W), 27, cin, cout, NV.ptr(wimg), nb, NV.stream()), "wimage")
        bn = NV.BnP(None, None, None, None)
        outs, res = {}, {}
        for ps in (0, 1):
            out = torch.empty(Mout, cout, device=dev)
            op = torch.zeros(Mout, 3, cout, dtype=torch.int16, device=dev)

            def go():
                NV.check(L.mvr_spconv_x(NV.ptr(x), cin, cin, NV.ptr(nbr), NV.ptr(perm), 27, Mout, NV.ptr(W), cout,
                                        None, bn, 1e-5, None, 0, 1, NV.ptr(out), cout, NV.ptr(wimg), None,
                                        NV.ptr(xp) if ps else None, NV.ptr(op) if ps else None, NV.stream()),
                         "spconv_x")
            for _ in range(2):
                go()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.iters):
                go()
            e1.record()
            torch.cuda.synchronize()
            res[ps] = e0.elapsed_time(e1) / a.iters
            outs[ps] = (out.clone(), op)
        same = torch.equal(outs[0][0], outs[1][0])
        psame = torch.equal(outs[1][1], planes(outs[1][0]))
        for ps in (0, 1):
            tot[ps] += res[ps]
        print("%-16s Mout %7d  fp32 gathers %.3f ms  pre-split %.3f ms  (%.2fx)  outputs bit-identical %s, "
              "out planes = torch split %s" % (tag, Mout, res[0], res[1], res[0] / res[1], same, psame), flush=True)
    print("total over the layer shapes: fp32 gathers %.3f ms, pre-split %.3f ms" % (tot[0], tot[1]), flush=True)


if __name__ == "__main__":
    main()
