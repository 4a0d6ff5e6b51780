"""Round 5: device timeline of a rocprofv3 kernel trace — per kernel name its count and mean
duration, then the last N DP kernels with the gap before each and what ran in it."""
import csv
import glob
import sys

path = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
rows.sort()
by = {}
for s, e, n in rows:
    by.setdefault(n, []).append(e - s)
for n, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    print("%-60s n %4d  mean %9.1f us" % (n[:60], len(d), sum(d) / len(d) / 1e3))
dps = [r for r in rows if "bg_dp_" in r[2]]
print("\nlast DP kernels: start (ms, from the first), duration, gap after the previous DP's end")
t0 = rows[0][0]
prev = None
for s, e, n in dps[-14:]:
    gap = (s - prev) / 1e6 if prev else 0.0
    inside = [x for x in rows if prev and prev <= x[0] < s and "bg_dp_" not in x[2]]
    what = ", ".join(sorted(set(x[2].replace("void ", "")[:28] for x in inside)))
    print("%9.3f  %7.3f ms  gap %7.3f ms  %s" % ((s - t0) / 1e6, (e - s) / 1e6, gap, what))
    prev = e
