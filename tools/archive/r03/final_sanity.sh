set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 2
timeout -k 10 500 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t14.log 2>&1; rc=$?; tail -2 gpurun_out/t14.log; exit $rc
