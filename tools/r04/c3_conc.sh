# round 4: C3 with the exit pass beside the DP (BG_SPLIT_CONC) and two DP streams
# (BG_TWO_DP_STREAMS), pipeline depths 3 and 4: pipelined and single-alignment walls
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/c3conc; export TMPDIR=/tmp
for p in 3 4; do
for v in "" "BG_SPLIT_CONC=1" "BG_TWO_DP_STREAMS=1" "BG_SPLIT_CONC=1 BG_TWO_DP_STREAMS=1"; do
  env $v X=1 timeout -k 10 200 python tools/configs.py C3 --steps 20 --single 5 --pipeline $p > gpurun_out/r04/c3conc/c3.txt 2>&1 || { echo "C3 [$v] p$p failed"; tail -5 gpurun_out/r04/c3conc/c3.txt; exit 4; }
  echo "p$p [$v] $(tail -1 gpurun_out/r04/c3conc/c3.txt)" | tee -a gpurun_out/r04/c3conc/all.txt
done
done
