# C5 (and C2) geometry sweep: GCUPS, DP / finish ms per (R, W)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
CFG=${CFG:-C5}
for rw in ${RWS:-0,0 2,4 4,2 4,4 4,6 8,2 8,4}; do
  IFS=, read -r RR WW <<< "$rw"
  timeout -k 10 200 python tools/configs.py $CFG --R $RR --waves $WW 2>&1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$rw', d['gcups'], d['ms_per_step'], d['dp_ms'], d['finish_ms'], d['R'], d['waves'])" || exit 1
done
