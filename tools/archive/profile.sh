# rocprofv3 kernel-trace summary of the bench workload (no PMC here: counters in tools/pmc.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu --steps 5 --warmup 1 ${BENCH_ARGS} > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err
rc=$?
find gpurun_out/prof -name "*.csv" | head -20
cat gpurun_out/prof/bench.json
exit $rc
