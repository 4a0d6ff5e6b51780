set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -m pytest tests -x -q -m gpu ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "exit $rc" >> gpurun_out/gpu_tests.log
tail -40 gpurun_out/gpu_tests.log
exit $rc
