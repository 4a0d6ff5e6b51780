# round 4: A/B of the walker's s_setprio 3 (BG_FIN_NOPRIO=1 keeps it at 0): C2, C4, C5 and the metric
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/prio; export TMPDIR=/tmp
for rep in 1 2; do for v in ${VARS:-"X=1" "BG_FIN_NOPRIO=1"}; do
  env $v timeout -k 10 200 python tools/configs.py C2 C4 C5 --steps 20 > gpurun_out/r04/prio/cfg.txt 2>&1 || { tail -5 gpurun_out/r04/prio/cfg.txt; exit 4; }
  echo "[$v] $(python3 -c "
import json,sys
for l in open('gpurun_out/r04/prio/cfg.txt'):
    if l.startswith('{'): d=json.loads(l); print(d['config'], d['gcups'], 'dp', d['dp_ms'], 'fin', d['finish_ms'], end=' | ')
")"
  env $v timeout -k 10 200 python bench.py --no-cpu --no-h2h --no-affine --configs "" > gpurun_out/r04/prio/m.json 2> gpurun_out/r04/prio/m.err || { tail -5 gpurun_out/r04/prio/m.err; exit 4; }
  echo "[$v] M $(python3 -c "import json; d=json.load(open('gpurun_out/r04/prio/m.json')); print(d['value'], d['ms_per_step'])")"
done; done
