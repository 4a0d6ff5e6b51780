# A/B of the score-only linear DP's geometry and profile form on the metric workload.
# CFGS="P,R,W ..." (P = BG_P32: 0 byte/SDWA, 1 dword; R = 0 / W = 0: the planner's choice);
# prints GCUPS, step ms, DP / finish kernel ms and the kernel config.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for cfg in ${CFGS:-0,8,16 1,8,8 0,0,0}; do
  IFS=, read -r P RR WW <<< "$cfg"
  BG_P32=$P timeout -k 10 120 python bench.py --no-cpu --no-h2h --no-gather --R $RR --waves $WW ${BENCH_ARGS} 2>gpurun_out/p32.err \
    | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$cfg', d['value'], d['ms_per_step'], r['kernel_ms'], r['finish_ms'], d['config']['kernel'], d['all_status_ok'])" || { tail -5 gpurun_out/p32.err; exit 1; }
done
