set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
BG_DP_TIMING=1 timeout -k 10 120 python tools/dp_timeline.py --pairs 1 --len 100000 > gpurun_out/tl_c3_w.txt 2>&1 || exit 3
grep -E "span|strip    0 |strip  312 " gpurun_out/tl_c3_w.txt | tail -3
