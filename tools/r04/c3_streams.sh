# round 4: C3 with the split traceback — two DP streams vs one, and the phase breakdown
# (rocprofv3 kernel stats of a C3 run)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/c3s; export TMPDIR=/tmp
timeout -k 10 300 python tools/configs.py C3 --steps 20 --single 5 > gpurun_out/r04/c3s/two_dp.txt 2>&1 || exit 4
tail -1 gpurun_out/r04/c3s/two_dp.txt
BG_ONE_DP_STREAM=1 timeout -k 10 300 python tools/configs.py C3 --steps 20 --single 5 > gpurun_out/r04/c3s/one_dp.txt 2>&1 || exit 5
tail -1 gpurun_out/r04/c3s/one_dp.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04/c3s/prof -o run --output-format csv -- python3 tools/configs.py C3 --steps 6 --single 3 > gpurun_out/r04/c3s/prof.txt 2> gpurun_out/r04/c3s/prof.err || { tail -5 gpurun_out/r04/c3s/prof.err; exit 6; }
f=$(find gpurun_out/r04/c3s/prof -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r04/c3s/kernel_stats_C3.csv
python3 - gpurun_out/r04/c3s/kernel_stats_C3.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-70s n %4s avg %10.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
