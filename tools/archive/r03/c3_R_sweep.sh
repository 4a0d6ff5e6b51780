set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for R in 2 3 4 5 8; do
  timeout -k 10 200 python tools/configs.py C3 --steps 12 --pipeline 4 --R $R > gpurun_out/c3_R$R.txt 2>&1 || exit 4
  echo R $R; tail -1 gpurun_out/c3_R$R.txt
done
for R in 3 4; do
  BG_DP_TIMING=1 timeout -k 10 120 python tools/dp_timeline.py --pairs 1 --len 100000 --R $R > gpurun_out/tl_c3_R$R.txt 2>&1 || exit 3
  grep -E "span" gpurun_out/tl_c3_R$R.txt | tail -1
done
