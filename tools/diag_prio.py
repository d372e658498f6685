"""Pipelined scene bench with other stream priorities (diagnostic): python tools/diag_prio.py <A> <B> <C> [bench args],
each 0 (normal) or -1 (high).  bench.py's choice: 0 -1 -1."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

pa, pb, pc = (int(v) for v in sys.argv[1:4])
orig = bench.SceneWorkload.step_pipelined


def step_pipelined(self, world):
    if not hasattr(self, "streams"):
        self.streams = tuple(torch.cuda.Stream(self.dev, priority=p) for p in (pa, pb, pc))
        self.pending = None
        self.prepared = None
        print("stream priorities A %d B %d C %d" % (pa, pb, pc), file=sys.stderr)
    return orig(self, world)


bench.SceneWorkload.step_pipelined = step_pipelined
sys.argv = [sys.argv[0]] + sys.argv[4:]
bench.main()
