"""Is the OANet result a function of the stream it runs on (workspace, priority) rather than of
concurrency?  Full scene; stage hashes of finish() on the default stream, alone on a side stream (default
and high priority), and pipelined.  usage: python tools/diag_stage5.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from lib import _native as NV  # noqa: E402


def main():
    dev = torch.device("cuda")
    wl = bench.SceneWorkload(dev, 0)
    L = NV.lib()
    res = {}

    def run(tag, stream=None):
        with torch.no_grad():
            fin = wl.describe()
            torch.cuda.synchronize()
            buf = torch.zeros(256, dtype=torch.int64, device=dev)
            L.mvr_debug_stage_hash(NV.ptr(buf), 256)
            if stream is None:
                wl.finish(fin)
            else:
                with torch.cuda.stream(stream):
                    wl.finish(fin)
            torch.cuda.synchronize()
            L.mvr_debug_stage_hash(None, 0)
        res.setdefault(tag, []).append(buf.tolist())

    s0 = torch.cuda.Stream(dev)
    s1 = torch.cuda.Stream(dev, priority=-1)
    for _ in range(3):
        run("default")
    for _ in range(3):
        run("side", s0)
    for _ in range(3):
        run("side_hiprio", s1)
    for _ in range(2):
        run("default")
    ref = res["default"][1]
    n = max(i for i, v in enumerate(ref) if v) + 1
    for tag, hl in res.items():
        print(tag, [next((i for i in range(n) if h[i] != ref[i]), None) for h in hl], flush=True)


if __name__ == "__main__":
    main()
