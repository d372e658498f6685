"""Voxelise the bench's synthetic scene (30 fragments x 250 k raw points) repeatedly, for rocprofv3 kernel stats of
the voxelisation kernels (MVR_LIB selects a variant build)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "3d_multiview_reg_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden"))
import torch
from synth import synth_scene_fragments
from lib import sparse
from lib.sparse import fragment_views

dev = torch.device("cuda:0")
frags, _ = synth_scene_fragments(30, seed=41)
raw = fragment_views(frags, dev)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for r in range(reps):
    c, sel, counts, _ = sparse.voxelize(raw, 0.025, dev)
torch.cuda.synchronize()
t = time.time()
for r in range(reps):
    c, sel, counts, _ = sparse.voxelize(raw, 0.025, dev)
torch.cuda.synchronize()
print(f"voxelize {(time.time() - t) / reps * 1e3:.3f} ms per call (host-synchronising), {c.shape[0]} voxels, "
      f"lib {os.environ.get('MVR_LIB', 'default')}")
