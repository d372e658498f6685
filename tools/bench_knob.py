"""bench.py with library knobs set first (A/B timing):
  python tools/bench_knob.py <mvr_set_fn> <int> [bench args]
  python tools/bench_knob.py <mvr_set_fn>=<int>[,<mvr_set_fn>=<int>...] [bench args]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (sets up the package path)
from lib import _native  # noqa: E402

if "=" in sys.argv[1]:
    knobs = [(kv.split("=")[0], int(kv.split("=")[1])) for kv in sys.argv[1].split(",")]
    rest = sys.argv[2:]
else:
    knobs = [(sys.argv[1], int(sys.argv[2]))]
    rest = sys.argv[3:]
for fn, val in knobs:
    prev = getattr(_native.lib(), fn)(val)
    print("%s(%d) (was %d)" % (fn, val, prev), file=sys.stderr)
sys.argv = [sys.argv[0]] + rest
bench.main()
