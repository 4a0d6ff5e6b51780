# Profiles of the current build, as the bench runs it (pipeline depth 3):
#  1. rocprofv3 --kernel-trace --stats of the default bench (M, MA and the C2-C5 legs);
#  2. PMC passes (one counter group per pass, kernel trace only) for M, MA, C2, C3, C4, C5, each
#     summarised into profiles/pmc_<workload>.json by tools/pmc_traffic.py.
# Stops at the first failing GPU step.   TAG=r03 bash tools/prof_all.sh
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
TAG=${TAG:-run}; OUT=gpurun_out/prof_$TAG; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
  python3 bench.py --no-cpu --no-h2h --steps 20 --warmup 5 > $OUT/bench_under_rocprof.json 2> $OUT/stats.err \
  || { tail -5 $OUT/stats.err; exit 1; }
echo "stats ok"
G1="SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
METHOD="rocprofv3 --kernel-trace --pmc, one counter group per pass ($G1 | FETCH_SIZE | WRITE_SIZE), pipeline depth 3 as timed; averages over the DP dispatches"
for leg in ${LEGS:-M MA C2 C3 C4 C5}; do
  case $leg in
    M)  CMD="bench.py --no-cpu --no-h2h --no-affine --no-steady --configs= --steps 6 --warmup 2"; WL=semiglobal_256x10000x10000_blosum62_o1_e2 ;;
    MA) CMD="bench.py --no-cpu --no-h2h --no-affine --no-steady --configs= --steps 6 --warmup 2 --open -11 --extend -1"; WL=semiglobal_256x10000x10000_blosum62_o11_e1 ;;
    *)  CMD="tools/configs.py $leg --steps 4"; WL=$leg ;;
  esac
  i=0; mkdir -p $OUT/pmc_$leg
  for grp in "$G1" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmc_$leg/p$i -o run --output-format csv -- \
      python3 $CMD > $OUT/pmc_$leg/p$i.json 2> $OUT/pmc_$leg/p$i.err || { tail -5 $OUT/pmc_$leg/p$i.err; echo "pass $leg/$i failed"; exit 1; }
  done
  python3 tools/pmc_summary.py $OUT/pmc_$leg > /dev/null && python3 tools/pmc_traffic.py $OUT/pmc_$leg $WL $OUT/pmc_$leg/p1.json "$METHOD" || exit 1
done
mkdir -p $OUT/pmcout && cp profiles/pmc_*.json $OUT/pmcout/
find $OUT -name "*kernel_stats.csv"
