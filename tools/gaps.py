"""Idle gaps between kernels of one profiled step (rocprofv3 --kernel-trace csv): where the device
waits on the host.  usage: python tools/gaps.py <trace_kernel_trace.csv> [min_gap_us]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "vox_keys" in r["Kernel_Name"]]
s, e = idx[-2], idx[-1]
t0 = int(rows[s]["Start_Timestamp"])
prev = int(rows[s]["End_Timestamp"])
gaps, busy = 0.0, (prev - t0) / 1e3
for r in rows[s + 1:e]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = (st - prev) / 1e3
    if g > thr:
        print("%9.1f gap %7.1f us before %s" % ((st - t0) / 1e3, g, r["Kernel_Name"][:70]))
    gaps += max(g, 0.0)
    busy += (en - st) / 1e3
    prev = max(prev, en)
print("step span %.1f us, kernels %.1f us, gaps %.1f us, %d dispatches" % ((prev - t0) / 1e3, busy, gaps, e - s))
