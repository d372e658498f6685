"""Join rocprofv3 PMC passes (tools/pmc_bench.sh) with the bench's per-launch class sequence:
measured HBM bytes per launch for every kernel class of the timed step.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half the bytes of
16-byte-per-lane streaming reads (x2 here); WRITE_SIZE is exact for 16 B/lane stores; both in KB.
usage: python tools/pmc_traffic.py <outdir> [--out profiles/pmc_traffic.json]"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

NAME2CLASS = {"feat_nn_kernel": "feat_nn", "spconv_kernel": "spconv", "spconv_c1_kernel": "spconv",
              "procrustes_kernel": "procrustes"}
GEMM_CLASSES = ("conv_pts", "embed", "pool", "unpool", "oafilter")


def dispatches(d, counter):
    rows = {}
    for f in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = int(r["Dispatch_Id"])
            if k not in rows:
                rows[k] = [r["Kernel_Name"], 0.0]
            rows[k][1] += float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


def attribute(disp, seq):
    """-> {class: [bytes...]} for the timed step: GEMM dispatches joined to the sequence in order,
    other profiled kernels by name."""
    out = defaultdict(list)
    # launch_gemm's launches (gemm_kernel, or pconv_kernel for the 128 -> 128 point convs) in launch order
    gemm = [v for n, v in disp if "gemm_kernel" in n or "pconv_kernel" in n]
    seq_g = [c for c, _ in seq if c in GEMM_CLASSES]
    for c, v in zip(seq_g, gemm[len(gemm) - len(seq_g):]):
        out[c].append(v)
    n_other = defaultdict(int)
    for c, _ in seq:
        if c not in GEMM_CLASSES:
            n_other[c] += 1
    for key, cls in NAME2CLASS.items():
        vals = [v for n, v in disp if key + "<" in n or key + "(" in n]
        k = n_other.get(cls, 0)
        if k:
            out[cls].extend(vals[len(vals) - k:] if cls != "spconv" else vals[-k:])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = {}
    seq = json.load(open(os.path.join(a.outdir, "seq_FETCH_SIZE.json")))
    alg = defaultdict(list)
    for c, b in seq:
        alg[c].append(b)
    fetch = attribute(dispatches(a.outdir, "FETCH_SIZE"), seq)
    write = attribute(dispatches(a.outdir, "WRITE_SIZE"), json.load(open(os.path.join(a.outdir, "seq_WRITE_SIZE.json"))))
    for c in sorted(set(fetch) | set(write)):
        n = max(len(fetch[c]), len(write[c]), 1)
        fb = 2.0 * 1024 * sum(fetch[c]) / max(len(fetch[c]), 1)
        wb = 1024.0 * sum(write[c]) / max(len(write[c]), 1)
        ab = sum(alg[c]) / max(len(alg[c]), 1)
        res[c] = {"launches": n, "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                  "pmc_bytes_per_launch": fb + wb, "algorithmic_bytes_per_launch": ab,
                  "pmc_over_algorithmic": (fb + wb) / ab if ab else None}
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of `bench.py --steps 1 --warmup 1` "
                     "(tools/pmc_bench.sh); FETCH x2 (gfx950 16 B/lane correction), KB -> B",
           "classes": res}
    txt = json.dumps(doc, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
