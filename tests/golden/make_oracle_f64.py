#!/usr/bin/env python3
"""fp64 companions of reference fixtures, computed by OUR restatement (oracle/oanet.py in float64), not by the
reference: they measure how far the reference's own fp32 result sits from exact arithmetic on each pair, so a
parity test can tell rounding noise of a chaotic random network from a wrong result.

  oanet_full_train_f64.npz: oracle float64 forward of oanet_full_train.npz's inputs (train-mode BN, RegBlock
                            network, weights synth_state(seed 7), xs synth_correspondences(32, 5000, seed=33))

Usage: python tests/golden/make_oracle_f64.py   (~2 min on 8 cores)"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, ROOT]
from synth import synth_state, synth_correspondences  # noqa: E402
from oracle.oanet import oanet_forward  # noqa: E402


def main():
    with open(os.path.join(HERE, "oanet_keys.json")) as f:
        shapes = json.load(f)["full"]
    xs, _, _ = synth_correspondences(32, 5000, seed=33)
    o = oanet_forward(synth_state(shapes, seed=7), xs, train=True, dtype=np.float64)
    out = {}
    for i in range(2):
        out["R%d" % i] = o["rot_est"][i]
        out["t%d" % i] = o["trans_est"][i]
    np.savez_compressed(os.path.join(HERE, "oanet_full_train_f64.npz"), **out)
    print("wrote oanet_full_train_f64.npz")


if __name__ == "__main__":
    main()
