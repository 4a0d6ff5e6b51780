"""Turn a PMC pass set (tools/prof_all.sh) into profiles/pmc_<workload>.json (read by bench.py).

HBM bytes per DP launch = WRITE_SIZE*1024 + 2*FETCH_SIZE*1024: both rocprofv3 derived counters are
in KiB; on gfx950 FETCH_SIZE tallies 128-B read requests at 64 B (MI355X_MICROARCH.md, HBM
section), hence the factor 2 on reads.  WRITE_SIZE counts the EA write requests at their size.
The algorithmic bytes and the geometry come from the profiled run's own JSON line (bench.py's
roofline or tools/configs.py's algorithmic_bytes).

    python tools/pmc_traffic.py PASS_DIR WORKLOAD RUN_JSON METHOD
"""
import json
import sys

summ = json.load(open(sys.argv[1] + "/summary.json"))
workload = sys.argv[2]
line = json.loads([x for x in open(sys.argv[3]).read().splitlines() if x.startswith("{")][-1])
if "roofline" in line:
    algo = float(line["roofline"]["algorithmic_bytes_per_launch"])
    geom = [str(line["config"]["kernel"]["R"]), str(line["config"]["kernel"]["waves"])]
else:
    algo = float(line["algorithmic_bytes"])
    geom = [str(line["R"]), str(line["waves"])]
dp = {k: v for k, v in summ.items() if "dp" in k and "kernel" in k}
assert len(dp) == 1, list(summ)
name, c = next(iter(dp.items()))
write_b = c["WRITE_SIZE"] * 1024.0
fetch_b = c["FETCH_SIZE"] * 1024.0 * 2.0
fin = {k: v for k, v in summ.items() if "finish" in k}
out = {
    "workload": workload,
    "kernel": name,
    "geometry": geom,
    "write_bytes_per_launch": write_b,
    "fetch_bytes_per_launch_corrected": fetch_b,
    "fetch_size_kib_raw": c["FETCH_SIZE"],
    "write_size_kib_raw": c["WRITE_SIZE"],
    "hbm_bytes_per_launch": write_b + fetch_b,
    "algorithmic_bytes_per_launch": algo,
    "traffic_over_algorithmic": (write_b + fetch_b) / algo,
    "raw_counters": c,
    "finish_kernel_counters": fin,
    "method": sys.argv[4],
}
if c.get("SQ_WAVE_CYCLES"):
    out["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
    out["active_inst_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
print(json.dumps({k: v for k, v in out.items() if k not in ("raw_counters", "finish_kernel_counters")}))
with open("profiles/pmc_%s.json" % workload, "w") as f:
    json.dump(out, f, indent=1)
