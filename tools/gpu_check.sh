# GPU check of the current tree: every GPU test, then the default bench (configs legs included, no
# CPU leg).  usage (on the box): bash tools/gpu_check.sh <outdir under gpurun_out>
# PYTEST_K filters the tests, BENCH_ARGS adds bench flags, NO_TESTS=1 skips the tests,
# N2=1 adds a two-rank gloo rehearsal of the N > 1 bench (ranks share the GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-check}; mkdir -p $O; export TMPDIR=/tmp
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/gpu_tests.log 2>&1
  rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -20; exit $rc; }
fi
timeout -k 10 400 python bench.py --no-cpu ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 tools/summ_bench.py $O/bench.json
if [ -n "$N2" ]; then
  BG_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 6 --warmup 2 --no-h2h > $O/n2.json 2> $O/n2.err || { tail -20 $O/n2.err; exit 1; }
  python3 tools/summ_bench.py $O/n2.json
  BG_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 3 --warmup 1 --config C4 > $O/n2_c4.json 2> $O/n2_c4.err || { tail -20 $O/n2_c4.err; exit 1; }
  python3 tools/summ_bench.py $O/n2_c4.json
fi
