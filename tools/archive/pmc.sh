# rocprofv3 PMC passes over the bench workload (one counter group per pass, kernel trace only).
# Usage: PASSES="SQ_WAVES,SQ_INSTS_VALU;FETCH_SIZE" BENCH_ARGS="--R 10 --waves 16" bash tools/pmc.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
IFS=';' read -ra P <<< "${PASSES}"
i=0
for grp in "${P[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc ${grp//,/ } -d $OUT/p$i -o run --output-format csv -- python3 bench.py --no-cpu --steps 2 --warmup 0 --pipeline 1 ${BENCH_ARGS} > $OUT/p$i.json 2> $OUT/p$i.err || { tail -3 $OUT/p$i.err; echo "pass $i failed: $grp"; continue; }
  echo "pass $i: $grp ok"
done
python3 tools/pmc_summary.py $OUT
