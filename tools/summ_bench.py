"""One-screen summary of a bench.py JSON line (tools/gpu_check.sh)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("%s: %.1f GCUPS  %.4f ms/step  DP %.3f  fin %.3f  frac %.4f  status %s" % (
    d["config"]["workload"][:40], d["value"], d["ms_per_step"], r["kernel_ms"], r.get("finish_ms", 0),
    r["frac"], d["all_status_ok"]))
for k in ("affine", "strong", "pipelined_no_gather"):
    if d.get(k):
        print("  %s: %s GCUPS  %s ms/step" % (k, d[k]["value"], d[k]["ms_per_step"]))
for name, c in (d.get("configs") or {}).items():
    print("  %s: %.1f GCUPS  %.3f ms/step  DP %.3f  fin %.3f  R %d W %d  frac %.4f  ok %s  s4 %d" % (
        name, c["value"], c["ms_per_step"], c["dp_ms"], c["finish_ms"], c["kernel"]["R"],
        c["kernel"]["waves"], c["roofline"]["frac"], c["all_status_ok"], c["status4"]))
h = d.get("host_to_host")
if h:
    print("  h2h: %s GCUPS  %s s/batch  threads %s  phases %s" % (
        h["gcups"], h["seconds_per_batch"], h.get("host_threads"), h.get("host_ms_per_batch")))
if d.get("gather_ms") is not None:
    print("  gather_ms", d["gather_ms"])
