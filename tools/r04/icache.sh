# round 4: instruction-cache counters of the C4 kernels (one pass)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/icache; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES SQ_INSTS_SALU -d gpurun_out/r04/icache/p -o c4 --output-format csv -- python3 tools/configs.py C4 --steps 2 > gpurun_out/r04/icache/run.txt 2>&1 || { tail -5 gpurun_out/r04/icache/run.txt; exit 4; }
f=$(find gpurun_out/r04/icache/p -name "*counter_collection.csv" | head -1); echo "$f"
python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:60]; agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, {c: int(x) for c, x in v.items()})
PY
