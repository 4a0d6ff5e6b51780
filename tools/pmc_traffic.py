"""Turn a tools/pmc.sh summary into profiles/pmc_<workload>.json (read by bench.py).

HBM bytes per DP launch = WRITE_SIZE*1024 + 2*FETCH_SIZE*1024: both rocprofv3 derived counters are
in KiB; on gfx950 FETCH_SIZE tallies 128-B read requests at 64 B (MI355X_MICROARCH.md, HBM
section), hence the factor 2 on reads.  WRITE_SIZE counts the EA write requests at their size.

    python tools/pmc_traffic.py gpurun_out/pmc/summary.json WORKLOAD ALGO_BYTES [R W]
"""
import json
import sys

summ = json.load(open(sys.argv[1]))
workload = sys.argv[2]
algo = float(sys.argv[3])
dp = {k: v for k, v in summ.items() if "dp" in k and "kernel" in k}
assert len(dp) == 1, list(summ)
name, c = next(iter(dp.items()))
write_b = c["WRITE_SIZE"] * 1024.0
fetch_b = c["FETCH_SIZE"] * 1024.0 * 2.0
out = {
    "workload": workload,
    "kernel": name,
    "geometry": sys.argv[4:6],
    "write_bytes_per_launch": write_b,
    "fetch_bytes_per_launch_corrected": fetch_b,
    "fetch_size_kib_raw": c["FETCH_SIZE"],
    "write_size_kib_raw": c["WRITE_SIZE"],
    "hbm_bytes_per_launch": write_b + fetch_b,
    "algorithmic_bytes_per_launch": algo,
    "traffic_over_algorithmic": (write_b + fetch_b) / algo,
    "raw_counters": c,
    "method": "rocprofv3 --kernel-trace --pmc, one counter group per pass (tools/pmc.sh), "
              "bench.py --pipeline 1 --steps 2 --warmup 0; averages over the DP dispatches",
}
print(json.dumps(out, indent=1))
with open("profiles/pmc_%s.json" % workload, "w") as f:
    json.dump(out, f, indent=1)
