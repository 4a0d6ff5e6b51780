# round 4: traceback workgroups reserved beside the DP's per CU (BG_FIN_RESERVE) on C2, C4, C5
# (the BG_FIN_RESERVE knob was removed after this experiment: profiles/r04/geometry/fin_reserve_planner.txt)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/finres; export TMPDIR=/tmp
for k in 1 2 3 4 6; do
  BG_FIN_RESERVE=$k BG_PLAN_DEBUG= timeout -k 10 200 python tools/configs.py C2 C4 C5 --steps 20 > gpurun_out/r04/finres/cfg.txt 2>&1 || { tail -5 gpurun_out/r04/finres/cfg.txt; exit 4; }
  echo "[k=$k] $(python3 -c "
import json
for l in open('gpurun_out/r04/finres/cfg.txt'):
    if l.startswith('{'): d=json.loads(l); print(d['config'], d['gcups'], 'R', d['R'], 'W', d['waves'], 'dp', d['dp_ms'], 'fin', d['finish_ms'], 'bad', d['bad_status'], end=' | ')
")"
done
