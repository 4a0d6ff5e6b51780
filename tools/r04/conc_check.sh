# round 4: the exit pass beside the DP and two WIDE DP streams — parity first, then C3 timings
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/conc; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r04/conc/t_split.log 2>&1; rc=$?; tail -28 gpurun_out/r04/conc/t_split.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
for v in "" "BG_SPLIT_CONC=1" "BG_TWO_DP_STREAMS=1" "BG_SPLIT_CONC=1 BG_TWO_DP_STREAMS=1"; do
  env $v X=1 timeout -k 10 300 python tools/configs.py C3 --steps 20 --single 5 > gpurun_out/r04/conc/c3.txt 2>&1 || { echo "C3 [$v] failed"; tail -5 gpurun_out/r04/conc/c3.txt; exit 4; }
  echo "[$v] $(tail -1 gpurun_out/r04/conc/c3.txt)"
done
