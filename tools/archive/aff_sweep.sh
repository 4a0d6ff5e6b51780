# MA (256 x 10k x 10k semiglobal -11/-1) geometry sweep through bench.py: GCUPS, DP / finish ms
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rw in ${RWS:-0,0 2,8 2,16 4,4 4,8 4,16 8,8 8,16}; do
  IFS=, read -r RR WW <<< "$rw"
  timeout -k 10 120 python bench.py --no-cpu --no-h2h --no-affine --steps ${STEPS:-4} --warmup 1 \
    --open ${OPEN:--11} --extend ${EXT:--1} --R $RR --waves $WW ${BENCH_ARGS} > gpurun_out/sw.json 2> gpurun_out/sw.err \
    || { tail -3 gpurun_out/sw.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sw.json')); k=d['config']['kernel']; r=d['roofline']; print('$rw', d['value'], d['ms_per_step'], r['kernel_ms'], r['finish_ms'], k['R'], k['waves'], d['all_status_ok'])"
done
