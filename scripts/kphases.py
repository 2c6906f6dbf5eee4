"""Spill / instruction census of one kernel's ISA between its s_memtime stamp markers.
    python scripts/kphases.py /tmp/isa/<file>.s <kernel-symbol-prefix>"""
import re
import sys
from collections import Counter

path, sym = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(sym) and l.rstrip().endswith(":") is False or l.startswith(sym + ":") or (l.startswith(sym) and ":" in l))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
seg, phase = Counter(), 0
rows = []
for l in lines[start:end + 1]:
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    op = t.split()[0]
    if op == "s_memtime":
        rows.append((phase, seg)); seg = Counter(); phase += 1
        continue
    seg[op] += 1
rows.append((phase, seg))
for ph, c in rows:
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print("segment %2d: %5d instrs, VALU %5d, f64 %4d, scratch ld %3d st %3d, ds %3d, barrier %d" % (
        ph, sum(c.values()), valu, sum(v for k, v in c.items() if "f64" in k),
        sum(v for k, v in c.items() if k.startswith("scratch_load")),
        sum(v for k, v in c.items() if k.startswith("scratch_store")),
        sum(v for k, v in c.items() if k.startswith("ds_")), c["s_barrier"]))
