"""Summarise rocprofv3 --pmc CSVs (per kernel name: mean of each counter over dispatches)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "p*", "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"][:60]
            acc[k][row["Counter_Name"]].append((int(row["Dispatch_Id"]), float(row["Counter_Value"])))
    out = {}
    for k, cs in acc.items():
        o = {}
        for c, vals in cs.items():
            per = defaultdict(float)
            for did, v in vals:
                per[did] += v            # sum over dimensions (XCD/SE instances) of one dispatch
            o[c] = sum(per.values()) / len(per)
        out[k] = o
    return out


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print("==", d)
        for k, o in load(d).items():
            print(" ", k)
            for c in sorted(o):
                print("    %-28s %.4g" % (c, o[c]))
