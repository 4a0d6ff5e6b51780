set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for ch in 1 400 800 1200; do
  BG_DP_TIMING=$ch timeout -k 10 120 python tools/dp_timeline.py --pairs 1 --len 100000 > gpurun_out/tl_ch$ch.txt 2>&1 || exit 3
done
echo ok
