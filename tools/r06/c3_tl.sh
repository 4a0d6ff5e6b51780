# Round 6: C3's strip chain — per-wave boundary arrival / departure times of the first twelve half
# boundaries and two steady ones (BG_DEBUG=dp, tools/dp_timeline.py), then C3's single wall.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-r06/c3_tl}; mkdir -p $O; export TMPDIR=/tmp
BG_DEBUG=dp timeout -k 10 120 python3 tools/dp_timeline.py --pairs 1 --len 100000 ${TL_ARGS} > $O/tl.txt 2>&1 || { tail -20 $O/tl.txt; exit 1; }
grep -E "run 1|span" $O/tl.txt | tail -2
timeout -k 10 200 python3 tools/configs.py C3 --single 5 ${CFG_ARGS} > $O/c3.txt 2>&1 || { tail -20 $O/c3.txt; exit 2; }
tail -3 $O/c3.txt
if [ -n "$TESTS" ]; then
  if [ "$TESTS" = all ]; then T=tests; else T="tests/test_zz_gpu_c3_full.py tests/test_gpu_parity.py tests/test_gpu_span.py tests/test_gpu_split.py"; fi
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $T > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 3; }
  tail -2 $O/tests.txt
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python bench.py --no-cpu --configs '' --no-affine --no-h2h > $O/bench_m.json 2> $O/bench_m.err || { tail -20 $O/bench_m.err; exit 4; }
  python3 tools/summ_bench.py $O/bench_m.json
fi
