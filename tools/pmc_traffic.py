"""Join rocprofv3 PMC passes (tools/pmc_bench.sh) with the bench's per-launch class sequence:
measured HBM bytes per profiled launch for every kernel class of the timed step.

The bench runs with MVR_PROF_MARK=1, so the library brackets every profiled region (one entry of
the class sequence, `mvr_prof_seq`) with two empty marker dispatches (csrc/prof.hip).  A dispatch
between the k-th begin marker and its end marker belongs to the k-th region; dispatches outside
every region (torch glue, the warmup step, which runs before profiling is switched on and so emits
no markers) are not attributed.  The number of marker pairs must equal the sequence length.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half the bytes of
16-byte-per-lane streaming reads (x2 here); WRITE_SIZE is exact for 16 B/lane stores; both in KB.
usage: python tools/pmc_traffic.py <outdir> [--out profiles/pmc_traffic.json]"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

BEGIN, END = "mvr_prof_mark_begin_kernel", "mvr_prof_mark_end_kernel"


def dispatches(d, counter):
    """[(kernel name, counter value)] in dispatch order."""
    rows = {}
    for f in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = int(r["Dispatch_Id"])
            if k not in rows:
                rows[k] = [r["Kernel_Name"], 0.0]
            rows[k][1] += float(r["Counter_Value"])
    return [tuple(rows[k]) for k in sorted(rows)]


def attribute(disp, seq):
    """-> ({class: [value per region]}, {class: {kernel: n}}) by position between the region markers."""
    per_region = [0.0] * len(seq)
    kernels = [defaultdict(int) for _ in seq]
    stack, k = [], 0
    for name, v in disp:
        if BEGIN in name:
            assert k < len(seq), "more marked regions than sequence entries"
            stack.append(k)
            k += 1
        elif END in name:
            assert stack, "unbalanced region markers"
            stack.pop()
        elif stack:   # innermost open region
            per_region[stack[-1]] += v
            kernels[stack[-1]][name.replace("(anonymous namespace)::", "").split("(")[0]] += 1
    assert k == len(seq) and not stack, "marked regions (%d) != sequence entries (%d)" % (k, len(seq))
    out, names = defaultdict(list), defaultdict(lambda: defaultdict(int))
    for (cls, _), v, ks in zip(seq, per_region, kernels):
        out[cls].append(v)
        for n, c in ks.items():
            names[cls][n] += c
    return out, names


def lib_hash():
    """source identity of the library the passes ran (the same MVR_LIB the bench loads): bench.py prices a run with
    these counters only when its own library reports the same hash"""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3d_multiview_reg_amd"))
    from lib import _native
    return _native.source_hash()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--out", default=None)
    ap.add_argument("--math", default="f32eq", help="the bench's --math of the profiled run")
    a = ap.parse_args()
    res = {}
    seq_f = json.load(open(os.path.join(a.outdir, "seq_FETCH_SIZE.json")))
    seq_w = json.load(open(os.path.join(a.outdir, "seq_WRITE_SIZE.json")))
    assert [c for c, _ in seq_f] == [c for c, _ in seq_w], "the two passes ran different launch sequences"
    alg = defaultdict(list)
    for c, b in seq_f:
        alg[c].append(b)
    fetch, names = attribute(dispatches(a.outdir, "FETCH_SIZE"), seq_f)
    write, _ = attribute(dispatches(a.outdir, "WRITE_SIZE"), seq_w)
    for c in sorted(alg):
        n = len(alg[c])
        fb = 2.0 * 1024 * sum(fetch[c]) / n
        wb = 1024.0 * sum(write[c]) / n
        ab = sum(alg[c]) / n
        res[c] = {"launches": n, "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                  "pmc_bytes_per_launch": fb + wb, "algorithmic_bytes_per_launch": ab,
                  "pmc_over_algorithmic": (fb + wb) / ab if ab else None,
                  "kernels": dict(sorted(names[c].items()))}
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of `bench.py --steps 1 --warmup 1` with "
                     "MVR_PROF_MARK=1 (tools/pmc_bench.sh): dispatches joined to the timed step's launch sequence "
                     "by region markers; FETCH x2 (gfx950 16 B/lane correction), KB -> B",
           "math": a.math, "lib_hash": lib_hash(), "classes": res}
    txt = json.dumps(doc, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
