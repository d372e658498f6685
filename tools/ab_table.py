"""Summarise bench.py JSON lines from logs: step time, median, and the per-class ms (profiled sequential step).
usage: python tools/ab_table.py gpurun_out/bench*.log"""
import json
import sys

cls_order = ["conv_pts", "pool", "unpool", "oafilter", "feat_nn", "spconv", "sparse_misc", "procrustes"]
print("%-28s %8s %8s %8s  %s" % ("leg", "ms/step", "median", "value", "  ".join("%11s" % c for c in cls_order)))
for fn in sys.argv[1:]:
    line = None
    for ln in open(fn, errors="replace"):
        if ln.startswith("{\"metric\""):
            line = json.loads(ln)
    if line is None:
        print("%-28s (no result)" % fn)
        continue
    c = line.get("roofline", {}).get("classes", {})
    print("%-28s %8.3f %8.3f %8.0f  %s" % (fn.split("/")[-1][:28], line["ms_per_step"], line.get("ms_per_step_median", 0),
                                        line["value"], "  ".join("%11.3f" % c.get(k, [0])[0] for k in cls_order)))
