"""SURVEY §5 sanitizers on host code: the C restatement of the FCGF kernel maps and sparse conv (oracle/csrc/
sparse_conv.c, the CPU baseline's FCGF leg) built with -fsanitize=address,undefined (`make -C oracle sanitize`) and
run in a child process under the ASan runtime, on a real fragment, against the numpy restatement.  Any heap overflow,
use-after-free or undefined behaviour aborts the child (-fno-sanitize-recover=all).  (GPU sanitizers are not available
on this pool; the device code's bounds are covered by the GPU parity tests and the shape checks of each entry point.)"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys
import numpy as np
sys.path[:0] = [{root!r}, {golden!r}]
from synth import synth_scene_fragments, synth_state
from oracle import fcgf
frags, _ = synth_scene_fragments(1, seed=44, n_pts=12000)
c, _, _ = fcgf.voxelize(frags, 0.025)
fcgf.set_threads(1)
c2 = fcgf.downsample(c, 2)
t1, t2 = fcgf.Table(c), fcgf.Table(c2)
for oc, ic, tab, ks, step, tr in ((c, c, t1, 3, 1, False), (c, c, t1, 7, 1, False), (c2, c, t1, 3, 1, False),
                                  (c, c2, t2, 3, 1, True), (c2, c2, t2, 3, 2, False)):
    np.testing.assert_array_equal(fcgf.kernel_map_c(oc, ic, ks, step, tr), fcgf.kernel_map(oc, tab, ks, step, tr))
rng = np.random.default_rng(0)
nbr = fcgf.kernel_map(c, t1, 3, 1, False)
f = rng.standard_normal((len(c), 32)).astype(np.float32)
W = rng.standard_normal((27, 32, 64)).astype(np.float32)
b = rng.standard_normal(64).astype(np.float32)
np.testing.assert_allclose(fcgf.sparse_conv_c(f, nbr, W, b), fcgf.sparse_conv(f, nbr, W, b), rtol=1e-4, atol=1e-4)
print("sanitized ok", fcgf.isa())
'''


def _asan_runtime():
    r = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True)
    p = r.stdout.strip()
    return p if r.returncode == 0 and os.path.isabs(p) and os.path.exists(p) else None


def test_c_restatement_under_asan_and_ubsan():
    rt = _asan_runtime()
    if rt is None:
        pytest.skip("no libasan in this toolchain")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], check=True)
    env = dict(os.environ, LD_PRELOAD=rt, MVO_LIB=os.path.join(ROOT, "oracle", "build", "libmvoracle_asan.so"),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="1")
    code = CHILD.format(root=ROOT, golden=os.path.join(ROOT, "tests", "golden"))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "sanitized ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
