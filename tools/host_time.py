"""Host-side time of the pipelined scene step (how long the Python/ctypes enqueue and its host syncs
take) against the device step time.  usage: python tools/host_time.py [--steps 10]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--cprofile", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from lib import _native
    _native.lib()
    wl = bench.SceneWorkload(dev, 0)
    with torch.no_grad():
        for _ in range(3):
            wl.step_pipelined(1)
        torch.cuda.synchronize()
        tot0 = time.perf_counter()
        host, desc, fin, prep = [], [], [], []
        orig_describe, orig_finish, orig_prepare = wl.describe, wl.finish, wl.prepare

        def describe(data=None):
            t = time.perf_counter()
            r = orig_describe(data)
            desc.append(time.perf_counter() - t)
            return r

        def prepare():
            t = time.perf_counter()
            r = orig_prepare()
            prep.append(time.perf_counter() - t)
            return r

        def finish(f):
            t = time.perf_counter()
            r = orig_finish(f)
            fin.append(time.perf_counter() - t)
            return r
        wl.describe, wl.finish, wl.prepare = describe, finish, prepare
        for _ in range(a.steps):
            t = time.perf_counter()
            wl.step_pipelined(1)
            host.append(time.perf_counter() - t)
        torch.cuda.synchronize()
        tot = time.perf_counter() - tot0
    ms = lambda v: "%.2f" % (1e3 * sum(v) / len(v))  # noqa: E731
    print("per step: wall %.2f ms | host step_pipelined %s ms (describe %s, finish %s, prepare %s)"
          % (1e3 * tot / a.steps, ms(host), ms(desc), ms(fin), ms(prep)), flush=True)
    if a.cprofile:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        with torch.no_grad():
            pr.enable()
            for _ in range(5):
                wl.step_pipelined(1)
            pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
