# round 4: split traceback — parity tests, WIDE / C3 tests, C3 pipelined + single-execute timing
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r04/t_split.log 2>&1; rc=$?; tail -25 gpurun_out/r04/t_split.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_configs.py -k "wide or C3" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/t_wide.log 2>&1; rc=$?; tail -5 gpurun_out/r04/t_wide.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/configs.py C3 --steps 12 --single 5 > gpurun_out/r04/c3.txt 2>&1 || exit 4
tail -3 gpurun_out/r04/c3.txt
BG_SPLIT=0 timeout -k 10 300 python tools/configs.py C3 --steps 12 --single 3 > gpurun_out/r04/c3_nosplit.txt 2>&1 || exit 5
tail -3 gpurun_out/r04/c3_nosplit.txt
