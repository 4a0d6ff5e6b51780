# End-of-session validation: every GPU test, smoke, the bench at the driver's settings, rocprofv3
# kernel stats of the bench and of C3, the configs at 12 steps.  Stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/final
export TMPDIR=/tmp
O=gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['finish_ms'], 'MA', d['affine']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_bench -o run --output-format csv -- \
  python3 bench.py --no-cpu --no-h2h --steps 10 --warmup 2 > $O/bench_under_rocprof.json 2> $O/stats_bench.err || { tail -5 $O/stats_bench.err; exit 1; }
echo "bench stats ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c3 -o run --output-format csv -- \
  python3 tools/configs.py C3 --steps 4 > $O/c3_under_rocprof.json 2> $O/stats_c3.err || { tail -5 $O/stats_c3.err; exit 1; }
echo "C3 stats ok"
timeout -k 10 400 python tools/configs.py C2 C3 C4 C5 --steps 12 > $O/configs.jsonl 2>&1 || { tail -5 $O/configs.jsonl; exit 1; }
cat $O/configs.jsonl | cut -c1-200
find $O -name "*kernel_stats.csv"
