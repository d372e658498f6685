"""Instruction mix per basic block of one kernel in a hipcc -S listing (blocks holding MFMAs).
usage: python tools/asm_mix.py <file.s> <kernel-symbol-substring>"""
import re
import sys
from collections import Counter

src, sym = sys.argv[1], sys.argv[2]
lines, on = [], False
for ln in open(src):
    if ln.startswith(sym) or (not on and re.match(r"^\S*%s\S*:" % re.escape(sym), ln)):
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
    c = Counter(ins)
    if c["v_mfma_f32_32x32x16_bf16"] + c["v_mfma_f32_32x32x2_f32"] == 0:
        continue
    valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
    salu = sum(v for k, v in c.items() if k.startswith("s_"))
    print("%s: %d instrs, VALU %d, SALU %d, MFMA %d" % (name, len(ins), valu, salu,
          c["v_mfma_f32_32x32x16_bf16"] + c["v_mfma_f32_32x32x2_f32"]))
    print("   ", ", ".join("%s %d" % kv for kv in c.most_common(18)))
