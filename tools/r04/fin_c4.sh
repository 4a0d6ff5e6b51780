# round 4: C4 finish phases, end-cell keys on / off, pipeline 3 / 1
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/finc4; export TMPDIR=/tmp
for v in "X=1"; do for p in 3 1; do
  env $v BG_FINISH_TIMING=1 timeout -k 10 150 python tools/configs.py C4 --steps 2 --pipeline $p > gpurun_out/r04/finc4/c4.txt 2>&1 || { tail -5 gpurun_out/r04/finc4/c4.txt; exit 4; }
  echo "[$v p$p] $(grep 'finish timing' gpurun_out/r04/finc4/c4.txt | tail -3 | tr '\n' ' ')"
  echo "    $(tail -1 gpurun_out/r04/finc4/c4.txt | cut -c150-330)"
done; done
