# GPU tests (optionally -k), then C3 timing (configs.py) and its DP timeline
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 200 python tools/configs.py C3 --steps 2 ${CFG_ARGS} 2>&1 | tail -1 || exit 1
BG_DP_TIMING=1 timeout -k 10 200 python tools/dp_timeline.py --pairs 1 --len 100000 > gpurun_out/tl_c3.txt 2>&1 || exit 1
grep -E "run 1|span|wave +(0|256|512|768|781) " gpurun_out/tl_c3.txt | tail -7 | cut -c1-170
