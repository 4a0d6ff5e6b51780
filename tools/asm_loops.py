"""Summarise the hot basic blocks of a kernel in a hipcc --save-temps .s file.

    python tools/asm_loops.py FILE.s KERNEL_SUBSTRING [min_marker_count] [marker]
"""
import re
import sys
from collections import Counter

path, kname = sys.argv[1], sys.argv[2]
minc = int(sys.argv[3]) if len(sys.argv) > 3 else 100
marker = sys.argv[4] if len(sys.argv) > 4 else "v_alignbit"
s = open(path).read()
m = re.search(r"^(_Z\S*%s\S*):" % re.escape(kname), s, re.M)
start = m.start()
end = s.index(".Lfunc_end", start)
blocks, cur = [], []
for line in s[start:end].split("\n"):
    if re.match(r"^\.LBB\d+_\d+:", line) or re.match(r"^_Z", line):
        if cur:
            blocks.append(cur)
        cur = [line]
    else:
        cur.append(line)
blocks.append(cur)
for b in blocks:
    ins = [l.strip().split()[0] for l in b[1:]
           if l.strip() and not l.strip().startswith((".", ";", "//"))]
    n = sum(1 for x in ins if x.startswith(marker))
    if n >= minc:
        c = Counter(ins)
        print(b[0].split()[0], "instrs", len(ins), marker, n)
        print("  ", sorted(c.items(), key=lambda x: -x[1])[:32])
