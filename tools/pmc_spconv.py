"""Mean FETCH_SIZE per spconv launch for each (row order, xcd) variant of tools/pmc_spconv.sh's run, in the order
tools/spconv_micro.py issues them (2 warmup + iters launches each).  FETCH_SIZE is in KB; x2 is the guide's gfx950
correction for 16-byte-per-lane reads (the gathers are 16-byte loads).
usage: python tools/pmc_spconv.py <outdir> [iters]"""
import csv
import glob
import os
import sys

ORDERS = ["none", "mask", "mask+morton", "morton", "frag+mask", "cell12+mask", "cell15+mask"]


def main():
    d, iters = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows = {}
    for f in glob.glob(os.path.join(d, "FETCH_SIZE", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "FETCH_SIZE" and "spconv_bx_kernel" in r["Kernel_Name"]:
                k = int(r["Dispatch_Id"])
                rows[k] = rows.get(k, 0.0) + float(r["Counter_Value"])
    v = [rows[k] for k in sorted(rows)]
    per = 2 + iters
    print("variant             launches  FETCH_SIZE MB (raw)  x2 (gfx950 16 B/lane)")
    for i, o in enumerate(ORDERS):
        for x in (0, 1):
            j = (2 * i + x) * per
            sel = v[j + 2:j + per]
            if sel:
                m = sum(sel) / len(sel) / 1024.0
                print("%-18s  %8d  %18.1f  %10.1f" % ("%s/x%d" % (o, x), len(sel), m, 2 * m))


if __name__ == "__main__":
    main()
