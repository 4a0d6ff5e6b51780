# round 4: kernel trace of lone C3 executes (which kernels the 1.3 ms traceback consists of)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/c3trace; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r04/c3trace/p -o run --output-format csv -- python3 tools/configs.py C3 --steps 1 --single 4 --pipeline 1 > gpurun_out/r04/c3trace/run.txt 2>&1 || { tail -5 gpurun_out/r04/c3trace/run.txt; exit 4; }
f=$(find gpurun_out/r04/c3trace/p -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
last = rows[-40:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%-45s %9.3f %9.3f %8.3f" % (r["Kernel_Name"][:45], (s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6))
PY
