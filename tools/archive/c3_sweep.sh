# C3 (one 100k x 100k pair, WIDE) sweep over R and the WIDE wave count: GCUPS, DP / finish ms
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rw in ${RWS:-2,4 3,4 4,4 5,4 8,4 2,8 4,8 8,8}; do
  IFS=, read -r RR WW <<< "$rw"
  BG_WIDE_W=$WW timeout -k 10 200 python tools/configs.py C3 --steps ${STEPS:-2} --R $RR 2>&1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$rw', d['gcups'], d['ms_per_step'], d['dp_ms'], d['finish_ms'], d['R'], d['waves'])" || exit 1
done
