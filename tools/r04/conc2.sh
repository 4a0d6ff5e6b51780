# round 4: the exit pass beside the DP alone (bounded waits + abandon record), then two DP streams
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/conc2; export TMPDIR=/tmp
timeout -k 10 150 python -u -m pytest tests/test_gpu_split.py -x -v -s -k beside_dp --timeout 100 --timeout-method thread > gpurun_out/r04/conc2/t_beside.log 2>&1; rc=$?; tail -30 gpurun_out/r04/conc2/t_beside.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 170 python -u -m pytest tests/test_gpu_split.py -x -v -s -k two_dp --timeout 60 --timeout-method thread > gpurun_out/r04/conc2/t_two.log 2>&1; rc=$?; tail -12 gpurun_out/r04/conc2/t_two.log | cut -c1-200; exit $rc
