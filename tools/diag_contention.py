"""Which stream-A work slows the filtering stream in the pipelined scene step (diagnostic; results are NOT valid
registrations): python tools/diag_contention.py <none|fcgf|nn|all> [bench args].  'fcgf' replaces the descriptor
network by a fixed feature table (sampling + feature NN still run), 'nn' skips the feature NN (the first step's
matches are reused), 'all' both."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

mode = sys.argv[1]
orig_describe = bench.SceneWorkload.describe
cache = {}


def describe(self, data=None):
    if data is None:
        data = self.prepare()
    pw = self.model
    if mode in ("nn", "all") and "fin" in cache:
        return cache["fin"]
    if mode in ("fcgf", "all"):
        if "F0" not in cache:
            n = data["sinput0_F"].shape[0]
            cache["F0"] = torch.nn.functional.normalize(torch.randn(n + 100000, 32, device=self.dev), dim=1)
        F0 = cache["F0"][: data["sinput0_F"].shape[0]]
        import numpy as np
        np.random.seed(self.rng_seed)
        xyz_b, f_b = pw.sampler(data["pcd0"].float().contiguous(), F0, data["pts_list"])
        fin, _, _ = pw.match_samples(data, xyz_b, f_b, F0, torch.empty(F0.shape[0], 0, device=self.dev))
    else:
        fin = orig_describe(self, data)
    if mode in ("nn", "all"):
        cache["fin"] = fin
    return fin


if mode != "none":
    bench.SceneWorkload.describe = describe
sys.argv = [sys.argv[0]] + sys.argv[2:]
bench.main()
