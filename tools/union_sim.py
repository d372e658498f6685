"""Offset-union work of the sparse conv's row tiles at 128 / 64 / 32 rows (the per-wave skip estimate):
the s1 3^3 kernel map of a few synthetic fragments (oracle/fcgf.py, CPU), rows in the library's order (active-offset
mask, then fragment and Morton code), union of the masks per tile x tile rows / active (row, offset) pairs.
usage: python tools/union_sim.py [--frags 4]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frags", type=int, default=4)
    a = ap.parse_args()
    import fcgf as F
    from synth import synth_scene_fragments
    xyz, _ = synth_scene_fragments(n_frag=a.frags)
    coords, _, _ = F.voxelize(list(xyz), 0.025)
    nbr = F.kernel_map(coords, F.Table(coords), 3, 1)
    mask = ((nbr >= 0).astype(np.int64) << np.arange(27)).sum(1)
    c = coords.astype(np.int64)
    q = c[:, 1:] & 255
    mort = np.zeros(len(c), np.int64)
    for b in range(8):
        for ax in range(3):
            mort |= ((q[:, ax] >> b) & 1) << (3 * b + 2 - ax)
    mort |= (c[:, 0] & 127) << 25
    order = np.lexsort((mort, mask))
    m = mask[order]
    act = (nbr >= 0).sum(1)[order]
    print("rows %d, active offsets per row %.2f" % (len(m), act.mean()))
    for tm in (128, 64, 32):
        n = len(m) // tm * tm
        un = np.bitwise_or.reduce(m[:n].reshape(-1, tm), axis=1)
        cnt = np.array([bin(int(x)).count("1") for x in un])
        print("%3d-row tiles: union work / active pairs = %.3f" % (tm, cnt.sum() * tm / act[:n].sum()))


if __name__ == "__main__":
    main()
