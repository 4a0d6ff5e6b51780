#!/usr/bin/env python3
"""Per-strip table of a BG_DEBUG=dp timeline (tools/dp_timeline.py output): start / end lags,
durations and the split of waiting into data, flow-control and other (boundary) cycles."""
import re
import sys

rows = []
for l in open(sys.argv[1]):
    m = re.match(r'\s+wave\s+(\d+) strip\s+(\d+) start\s+([\d.]+) c0done\s+([\d.]+) end\s+([\d.]+) us\s+waited\s+(\d+) of\s+(\d+) cycles(?:\s+data\s+(\d+) flow\s+(\d+))?', l)
    if m:
        rows.append(tuple(float(x or 0) for x in m.groups()))
rows = rows[len(rows) // 2:]          # the second (warm) run
every = int(sys.argv[2]) if len(sys.argv) > 2 else 1
for r in rows:
    w, s, st, c0, en, wt, tot, da, fl = r
    if int(s) % every and int(s) != int(rows[-1][1]):
        continue
    print(f"s{int(s):4d} c0 {c0:7.1f} end {en:8.1f} dur {en - c0:7.1f} comp {(tot - wt) / 1e6:5.2f}M "
          f"wait {wt / 1e6:5.2f}M data {da / 1e6:5.2f}M flow {fl / 1e6:5.2f}M other {(wt - da - fl) / 1e6:5.2f}M")
