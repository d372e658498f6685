"""Per-launch counters of tools/pmc_spconv_ps.sh's run, by sparse-conv kernel variant (PS = 0 fp32 gathers, PS = 1
pre-split planes): means over each variant's launches (2 warmup + iters).  FETCH_SIZE / WRITE_SIZE in KB (FETCH x2:
the guide's gfx950 correction for 16-byte-per-lane reads).
usage: python tools/pmc_spconv_ps.py <outdir>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "spconv_bx_kernel" not in k:
                continue
            v = "PS=1" if k.split("<")[1].split(">")[0].replace(" ", "").endswith(",1") else "PS=0"
            acc[v][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(v, r["Counter_Name"])].add(r["Dispatch_Id"])
    rows = {}
    for v, cs in acc.items():
        rows[v] = {c: cs[c] / max(1, len(disp[(v, c)])) for c in cs}
    names = sorted({c for v in rows for c in rows[v]})
    print("%-28s %16s %16s" % ("counter (mean per launch)", "PS=0", "PS=1"))
    for c in names:
        print("%-28s %16.4g %16.4g" % (c, rows.get("PS=0", {}).get(c, float("nan")), rows.get("PS=1", {}).get(c, float("nan"))))
    print()
    for v in ("PS=0", "PS=1"):
        x = rows.get(v, {})
        if not x:
            continue
        g = lambda n: x.get(n, float("nan"))
        print("%s: VALU per MFMA %.2f, LDS per MFMA %.2f, MFMA busy / CU-busy %.3f, waits %.3f of wave cycles, "
              "beyond-L2 reads %.1f MB (x2 corrected), writes %.1f MB" % (
                  v, g("SQ_INSTS_VALU") / g("SQ_INSTS_MFMA"), g("SQ_INSTS_LDS") / g("SQ_INSTS_MFMA"),
                  g("SQ_VALU_MFMA_BUSY_CYCLES") / g("SQ_BUSY_CU_CYCLES") if g("SQ_BUSY_CU_CYCLES") else float("nan"),
                  g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES"), 2 * g("FETCH_SIZE") / 1024, g("WRITE_SIZE") / 1024))


if __name__ == "__main__":
    main()
