set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_configs.py -k "wide or C3" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_wide.log 2>&1; rc=$?; tail -5 gpurun_out/t_wide.log; [ $rc -eq 0 ] || exit $rc
BG_DP_TIMING=1 timeout -k 10 120 python tools/dp_timeline.py --pairs 1 --len 100000 > gpurun_out/tl_c3.txt 2>&1 || exit 3
timeout -k 10 200 python tools/configs.py C3 --steps 12 > gpurun_out/c3.txt 2>&1 || exit 4
tail -3 gpurun_out/c3.txt
timeout -k 10 200 python tools/configs.py C3 --steps 12 --pipeline 4 > gpurun_out/c3_p4.txt 2>&1 || exit 5
tail -3 gpurun_out/c3_p4.txt
