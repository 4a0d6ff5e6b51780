# round 4: finish-kernel phase breakdown (BG_FINISH_TIMING) for C2, C4, C5 and the metric
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/finph; export TMPDIR=/tmp
for c in C2 C4 C5; do
  BG_FINISH_TIMING=1 timeout -k 10 150 python tools/configs.py $c --steps 2 > gpurun_out/r04/finph/$c.txt 2>&1 || { tail -5 gpurun_out/r04/finph/$c.txt; exit 4; }
  echo "$c: $(grep 'finish timing' gpurun_out/r04/finph/$c.txt | tail -1)"
  echo "    $(tail -1 gpurun_out/r04/finph/$c.txt | cut -c1-400)"
done
