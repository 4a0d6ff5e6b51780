"""Summarise rocprofv3 --pmc CSVs: per-kernel average of each counter over dispatches."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for path in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            short = name.split("(")[0]
            acc[short][row["Counter_Name"]].append((row.get("Dispatch_Id"), float(row["Counter_Value"])))
summary = {}
for k, counters in acc.items():
    summary[k] = {}
    for c, vals in counters.items():
        per = defaultdict(float)
        for d, v in vals:
            per[d] += v
        summary[k][c] = sum(per.values()) / max(len(per), 1)
print(json.dumps(summary, indent=1))
with open(os.path.join(out, "summary.json"), "w") as f:
    json.dump(summary, f, indent=1)
