# round 4: two traceback streams for many-pair batches (BG_TWO_FIN_STREAMS=1) re-checked with the
# walker at priority 0: metric, C2, C4, C5
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/twofin; export TMPDIR=/tmp
for rep in 1 2; do for v in "X=1" "BG_TWO_FIN_STREAMS=1"; do
  env $v timeout -k 10 200 python bench.py --no-cpu --no-h2h --no-affine --configs "" > gpurun_out/r04/twofin/m.json 2> gpurun_out/r04/twofin/m.err || { tail -5 gpurun_out/r04/twofin/m.err; exit 4; }
  echo "[$v] M $(python3 -c "import json; d=json.load(open('gpurun_out/r04/twofin/m.json')); print(d['value'], d['ms_per_step'])")"
  env $v timeout -k 10 200 python tools/configs.py C2 C4 C5 --steps 20 > gpurun_out/r04/twofin/cfg.txt 2>&1 || { tail -5 gpurun_out/r04/twofin/cfg.txt; exit 4; }
  echo "[$v] $(python3 -c "
import json
for l in open('gpurun_out/r04/twofin/cfg.txt'):
    if l.startswith('{'): d=json.loads(l); print(d['config'], d['gcups'], end=' | ')
")"
done; done
