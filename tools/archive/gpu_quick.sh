# GPU parity tests (optionally -k filtered) then the metric bench without the CPU leg
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -30; exit $rc; }
timeout -k 10 200 python bench.py --no-cpu --no-h2h ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms'], r['finish_ms'], d['all_status_ok'])"
timeout -k 10 300 python tools/configs.py C2 C4 C5 C3 --check 2 > gpurun_out/configs.log 2>&1 || { tail -20 gpurun_out/configs.log; exit 1; }
cat gpurun_out/configs.log
