set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_configs.py -k "wide or C3" -x -q --timeout 200 --timeout-method thread > gpurun_out/t5.log 2>&1; rc=$?; tail -3 gpurun_out/t5.log; [ $rc -eq 0 ] || exit $rc
BG_DP_TIMING=1 timeout -k 10 120 python tools/dp_timeline.py --pairs 1 --len 100000 > gpurun_out/tl_c3_5.txt 2>&1 || exit 3
grep -E "span|strip    0 |strip    1 |strip  312 " gpurun_out/tl_c3_5.txt | tail -4
for d in 3 4; do
  timeout -k 10 200 python tools/configs.py C3 --steps 12 --pipeline $d > gpurun_out/c3_5_d$d.txt 2>&1 || exit 4
  tail -1 gpurun_out/c3_5_d$d.txt
done
BG_DP_TIMING=800 timeout -k 10 120 python tools/dp_timeline.py --pairs 1 --len 100000 > gpurun_out/tl_c3_5_ch800.txt 2>&1 || exit 5
