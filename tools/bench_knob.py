"""bench.py with one library knob set first (A/B timing):  python tools/bench_knob.py <mvr_set_fn> <int> [bench args]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (sets up the package path)
from lib import _native  # noqa: E402

fn, val = sys.argv[1], int(sys.argv[2])
prev = getattr(_native.lib(), fn)(val)
print("%s(%d) (was %d)" % (fn, val, prev), file=sys.stderr)
sys.argv = [sys.argv[0]] + sys.argv[3:]
bench.main()
