# Kernel-trace stats of the default bench (M + MA legs), then PMC passes for M and MA separately
# (one counter group per pass, kernel trace only).  Stops at the first failing GPU step.
#   TAG=r02 bash tools/prof_round.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-run}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
  python3 bench.py --no-cpu --no-h2h --steps 10 --warmup 2 ${BENCH_ARGS} > $OUT/bench_under_rocprof.json 2> $OUT/stats.err \
  || { tail -5 $OUT/stats.err; exit 1; }
echo "stats ok"
G1="SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for leg in M MA; do
  if [ $leg = M ]; then GAPS="--open -1 --extend -2"; else GAPS="--open -11 --extend -1"; fi
  i=0; mkdir -p $OUT/pmc_$leg
  for grp in "$G1" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmc_$leg/p$i -o run --output-format csv -- \
      python3 bench.py --no-cpu --no-h2h --no-affine --steps 2 --warmup 1 $GAPS ${BENCH_ARGS} \
      > $OUT/pmc_$leg/p$i.json 2> $OUT/pmc_$leg/p$i.err || { tail -5 $OUT/pmc_$leg/p$i.err; echo "pass $leg/$i failed"; exit 1; }
    echo "pass $leg/$i ok"
  done
  python3 tools/pmc_summary.py $OUT/pmc_$leg > /dev/null
done
find $OUT -name "*kernel_stats.csv"
