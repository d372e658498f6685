"""Print a rocprofv3 *kernel_stats.csv compactly: calls, total ms, avg us, share, short name.
usage: python tools/kstats.py <kernel_stats.csv> [steps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    n = r["Name"]
    n = n.replace("(anonymous namespace)::", "").replace("mvr::", "")
    n = n.split("(")[0] if not n.startswith("void") else n[5:].split("(")[0]
    print("%6d %9.3f ms/step %9.1f us %6.2f%%  %s" % (int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6 / steps,
                                                     float(r["AverageNs"]) / 1e3, float(r["Percentage"]), n[:70]))
