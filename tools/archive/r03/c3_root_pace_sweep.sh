set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for p in 0 1 2 4; do
  BG_WIDE_PACE=$p BG_DP_TIMING=1 timeout -k 10 120 python tools/dp_timeline.py --pairs 1 --len 100000 > gpurun_out/tl_c3_p$p.txt 2>&1 || exit 3
  echo pace $p; grep -E "span|strip    0 |strip  312 " gpurun_out/tl_c3_p$p.txt | tail -3
done
for p in 0 2; do for d in 3 4; do
  BG_WIDE_PACE=$p timeout -k 10 200 python tools/configs.py C3 --steps 12 --pipeline $d > gpurun_out/c3_pace${p}_d$d.txt 2>&1 || exit 4
  echo pace $p depth $d; tail -1 gpurun_out/c3_pace${p}_d$d.txt
done; done
