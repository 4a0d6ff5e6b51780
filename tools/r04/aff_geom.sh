# round 4: C2 / C5 strip height re-checked (R x W)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/affgeom; export TMPDIR=/tmp
for cfg in "C2 2 4" "C2 4 4" "C2 4 2" "C2 8 2" "C5 2 2" "C5 4 2" "C5 4 4" "C5 2 4"; do set -- $cfg
  timeout -k 10 200 python tools/configs.py $1 --steps 20 --R $2 --waves $3 > gpurun_out/r04/affgeom/cfg.txt 2>&1 || { tail -5 gpurun_out/r04/affgeom/cfg.txt; exit 4; }
  echo "[$cfg] $(python3 -c "
import json
for l in open('gpurun_out/r04/affgeom/cfg.txt'):
    if l.startswith('{'): d=json.loads(l); print(d['config'], d['gcups'], 'R', d['R'], 'W', d['waves'], 'dp', d['dp_ms'], 'fin', d['finish_ms'], 'bad', d['bad_status'], end=' | ')
")"
done
