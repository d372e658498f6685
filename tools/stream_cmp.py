"""Per-kernel device time per step: the untimed sequential step (stream 0) vs the pipelined timed steps
(streams 1, 2) of a `tools/prof_bench.sh` kernel trace.  usage: stream_cmp.py <trace_kernel_trace.csv> <steps>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2])
tot = collections.defaultdict(float)
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
    tot[(n, r["Stream_Id"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
names = sorted({k[0] for k in tot}, key=lambda n: -tot.get((n, "0"), 0))
print(f"{'kernel':48s} {'seq ms':>8s} {'A ms/st':>8s} {'B ms/st':>8s}")
s0 = s1 = s2 = 0.0
for n in names:
    a, b, c = tot.get((n, "0"), 0), tot.get((n, "1"), 0) / steps, tot.get((n, "2"), 0) / steps
    s0 += a; s1 += b; s2 += c
    if max(a, b, c) > 0.05:
        print(f"{n:48s} {a:8.3f} {b:8.3f} {c:8.3f}")
print(f"{'total':48s} {s0:8.3f} {s1:8.3f} {s2:8.3f}")
