# bench the metric workload over kernel geometries: CONFIGS="R:W R:W ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
for cfg in ${CONFIGS}; do
  R=${cfg%%:*}; W=${cfg##*:}
  timeout -k 10 300 python bench.py --no-cpu --steps ${STEPS:-5} --warmup 1 --R $R --waves $W ${BENCH_ARGS} > gpurun_out/sweep/b_${R}_${W}.json 2> gpurun_out/sweep/b_${R}_${W}.err || { tail -5 gpurun_out/sweep/b_${R}_${W}.err; exit 1; }
  echo "R=$R W=$W $(python3 tools/summ.py < gpurun_out/sweep/b_${R}_${W}.json)"
done
