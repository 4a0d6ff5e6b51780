# round 5, final: smoke, the whole GPU suite, the default bench, rocprofv3 kernel stats of it
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r05/final5; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05/final5/smoke.txt 2>&1 || { tail -5 gpurun_out/r05/final5/smoke.txt; exit 1; }
tail -1 gpurun_out/r05/final5/smoke.txt
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r05/final5/t_gpu.log 2>&1; rc=$?
grep -E "FAIL|passed|failed" gpurun_out/r05/final5/t_gpu.log | cut -c1-200 | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r05/final5/bench.json 2> gpurun_out/r05/final5/bench.err || { tail -20 gpurun_out/r05/final5/bench.err; exit 3; }
python3 tools/summ_bench.py gpurun_out/r05/final5/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/final5/stats -o run --output-format csv -- python3 bench.py --no-cpu --no-h2h --steps 20 --warmup 5 > gpurun_out/r05/final5/bench_under_rocprof.json 2> gpurun_out/r05/final5/stats.err || { tail -5 gpurun_out/r05/final5/stats.err; exit 4; }
echo "stats ok"
