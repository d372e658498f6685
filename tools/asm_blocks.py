"""Per-basic-block instruction counts of one kernel in a hipcc -S listing (blocks with >= 8 instructions).
usage: python tools/asm_blocks.py <file.s> <kernel-symbol-prefix>"""
import re
import sys
from collections import Counter

sym = sys.argv[2]
lines, on = [], False
for ln in open(sys.argv[1]):
    if re.match(r"^%s\S*:" % re.escape(sym), ln):
        on = True
    if on:
        lines.append(ln)
        if "s_endpgm" in ln:
            break
blocks, cur, name = [], [], "entry"
for ln in lines:
    m = re.match(r"^(\.LBB\w+):", ln)
    if m:
        blocks.append((name, cur))
        name, cur = m.group(1), []
        continue
    t = ln.split()
    if t and re.match(r"^[vsdgb][a-z_0-9]+$", t[0]):
        cur.append(re.sub(r"_e(32|64)$", "", t[0]))
blocks.append((name, cur))
for name, ins in blocks:
    if len(ins) < 8:
        continue
    c = Counter(ins)
    valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
    mf = sum(v for k, v in c.items() if k.startswith("v_mfma"))
    print("%-10s %4d instrs VALU %4d MFMA %3d | %s" % (name, len(ins), valu, mf,
                                                      ", ".join("%s %d" % kv for kv in c.most_common(8))))
