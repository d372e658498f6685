"""Per-step kernel times from a rocprofv3 kernel-stats CSV (sequential bench profile): name filter, ms per step."""
import csv, sys
path, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 11.0
pat = sys.argv[3:] or [""]
rows = list(csv.DictReader(open(path)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if any(p in r["Name"] for p in pat):
        print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step {int(r['Calls']):6d} calls "
              f"{float(r['AverageNs']) / 1e3:9.1f} us  {r['Name'][:100]}")
