# new config-shape parity tests (no -x: see every failure), then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_configs.py} -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_new.log 2>&1
rc=$?; tail -15 gpurun_out/gpu_new.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ -n "$FULL" ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc2=$?; tail -15 gpurun_out/gpu_tests.log
exit $rc2
