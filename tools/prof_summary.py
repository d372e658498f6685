"""Summarise a rocprofv3 --kernel-trace --stats SQLite output (rocpd) as the stats CSV the older text outputs gave.

usage: python tools/prof_summary.py <run_results.db> [out.csv] [steps]
Prints the top kernels (ms total, calls, average us, ms per step when `steps` is given) and writes the CSV
(Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs) when `out.csv` is given.
"""
import csv
import sqlite3
import sys


def main():
    db = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "-" else None
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end - start), min(end - start), max(end - start) "
                     "from kernels group by name order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    if out:
        with open(out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for n, k, s, lo, hi in rows:
                w.writerow([n, k, s, s / k, 100.0 * s / tot, lo, hi])
    print("total device time %.3f ms%s" % (tot / 1e6, " (%.3f per step)" % (tot / 1e6 / steps) if steps else ""))
    for n, k, s, lo, hi in rows[:45]:
        ps = " %7.3f/step" % (s / 1e6 / steps) if steps else ""
        print("%9.3f ms %5d x %8.1f us%s  %s" % (s / 1e6, k, s / k / 1e3, ps, n[:100]))


if __name__ == "__main__":
    main()
