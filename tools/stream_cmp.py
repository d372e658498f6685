"""Per-kernel device time per step by HIP stream of a `tools/prof_bench.sh` kernel trace: stream 0 = the
untimed sequential profiled step; the other streams = the pipelined steps (bench.py: C voxelisation, A FCGF +
matching, B OANet, in creation order).  usage: stream_cmp.py <trace_kernel_trace.csv> <pipelined steps>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2])
tot = collections.defaultdict(float)
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("mvr::", "")[:44]
    tot[(n, r["Stream_Id"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
sids = sorted({k[1] for k in tot}, key=int)
names = sorted({k[0] for k in tot}, key=lambda n: -sum(tot.get((n, s), 0) for s in sids))
print("%-44s %s" % ("kernel (ms; stream 0 = one sequential step, others per pipelined step)",
                    " ".join("%9s" % ("s%s" % s) for s in sids)))
sums = collections.Counter()
for n in names:
    v = [tot.get((n, s), 0) / (1 if s == "0" else steps) for s in sids]
    for s, x in zip(sids, v):
        sums[s] += x
    if max(v) > 0.05:
        print("%-44s %s" % (n, " ".join("%9.3f" % x for x in v)))
print("%-44s %s" % ("total", " ".join("%9.3f" % sums[s] for s in sids)))
