"""Run-to-run determinism of the point-conv kernel (csrc/pconv.hip via mvr_gemm_f32) at the scene shape,
alone and with other kernels running beside it on a second stream.  Prints, per case, how many runs
differ from the first and where (pair, row, column) the first differing element sits.
usage: python tools/pconv_stress.py [runs]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d_multiview_reg_amd"))
import torch  # noqa: E402
from lib import _native as NV  # noqa: E402

P, C = 435, 128
N = int(os.environ.get("PSTRESS_N", "5000"))
CASES = {   # name: (K, pro, bias, stats, res)   res 2: in place (the residual is the output buffer)
    "res_inplace": (C, 2, 1, 1, 2),
    "plain": (C, 0, 1, 0, 0),
    "pro_stats": (C, 2, 1, 1, 0),
    "res": (C, 2, 1, 1, 1),
    "k256_pro_stats": (2 * C, 2, 1, 1, 0),
    "k256_plain": (2 * C, 0, 1, 0, 0),
}


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    d = torch.device("cuda")
    g = torch.Generator(device=d).manual_seed(0)
    L = NV.lib()
    noise_s = torch.cuda.Stream(d)
    big = torch.randn(64 << 20, device=d, generator=g)
    mm = torch.randn(4096, 4096, device=d, generator=g)
    for name, (K, pro, bias, stats, res) in CASES.items():
        Nl = (N + 31) // 32 * 32
        A = torch.randn(C, K, device=d, generator=g) * 0.1
        B = torch.randn(P, K, Nl, device=d, generator=g)
        R = torch.randn(P, C, Nl, device=d, generator=g) if res else None
        bv = torch.randn(C, device=d, generator=g)
        sc = torch.rand(P, K, device=d, generator=g) + 0.5 if pro else None
        sh = torch.rand(P, K, device=d, generator=g) if pro else None
        nt = (N + 127) // 128
        outs = []
        for r in range(runs + 1):
            Y = torch.full((P, C, Nl), float("nan"), device=d)
            if res == 2:
                Y.copy_(R)
            st = torch.full((P, nt, C, 2), float("nan"), device=d) if stats else None
            if r > runs // 2:   # second half: other kernels on another stream meanwhile
                with torch.cuda.stream(noise_s):
                    for _ in range(3):
                        big.mul_(1.0000001)
                        torch.mm(mm, mm)
            rc = L.mvr_gemm_f32(C, N, K, P, NV.ptr(A), 0, K, NV.ptr(B), K * Nl, Nl, 0, NV.ptr(Y), C * Nl, Nl,
                                NV.ptr(Y if res == 2 else R), C * Nl, NV.ptr(bv), bias, NV.ptr(sc), NV.ptr(sh), K, 0, pro, NV.ptr(st), C,
                                0, stats, 1, NV.ptr(NV.flag_word()), NV.stream())
            assert rc == 0, rc
            torch.cuda.synchronize()
            outs.append((Y[..., :N].clone(), st.clone() if stats else None))
        y0, s0 = outs[0]
        msg = []
        for r, (y, s) in enumerate(outs[1:], 1):
            bad = (y != y0) & ~(torch.isnan(y) & torch.isnan(y0))
            nb = int(bad.sum())
            sb = 0 if s is None else int(((s != s0) & ~(torch.isnan(s) & torch.isnan(s0))).sum())
            if nb or sb:
                idx = bad.nonzero()[:3].tolist()
                msg.append("run %d%s: %d values, %d stats differ; first %s" % (r, " (noise)" if r > runs // 2 else "",
                                                                          nb, sb, idx))
        print("%-15s nan in output: %s; %s" % (name, bool(torch.isnan(y0).any()), "; ".join(msg) if msg else "all runs identical"),
              flush=True)


if __name__ == "__main__":
    main()
