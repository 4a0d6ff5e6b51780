# round 4: the metric's geometry re-checked after the walker-priority change (R x W)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/mgeom; export TMPDIR=/tmp
for g in "8 16" "10 16" "5 16" "8 16"; do set -- $g
  timeout -k 10 200 python bench.py --no-cpu --no-h2h --no-affine --configs "" --R $1 --waves $2 > gpurun_out/r04/mgeom/m.json 2> gpurun_out/r04/mgeom/m.err || { tail -5 gpurun_out/r04/mgeom/m.err; exit 4; }
  echo "R $1 W $2: $(python3 -c "import json; d=json.load(open('gpurun_out/r04/mgeom/m.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], 'dp', r.get('dp_ms'), 'fin', r.get('finish_ms'))")"
done
