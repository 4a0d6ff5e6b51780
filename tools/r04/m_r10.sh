# round 4: the metric's DP alone (pipeline 1) at R = 8 and R = 10 (W = 16)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/mr10; export TMPDIR=/tmp
for g in "8 1" "10 1" "8 3" "10 3"; do set -- $g
  timeout -k 10 200 python bench.py --no-cpu --no-h2h --no-affine --configs "" --R $1 --waves 16 --pipeline $2 > gpurun_out/r04/mr10/m.json 2> gpurun_out/r04/mr10/m.err || { tail -5 gpurun_out/r04/mr10/m.err; exit 4; }
  echo "R $1 pipeline $2: $(python3 -c "import json; d=json.load(open('gpurun_out/r04/mr10/m.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], 'dp', r.get('dp_ms'), 'fin', r.get('finish_ms'))")"
done
