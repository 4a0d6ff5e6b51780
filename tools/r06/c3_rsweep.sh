# Round 6: C3's strip height after the border-code change (one alignment's wall, --single 5).
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-r06/c3_rsweep}; mkdir -p $O; export TMPDIR=/tmp
for R in ${RS:-2 3 4 5 8}; do
  timeout -k 10 200 python3 tools/configs.py C3 --single 5 --R $R > $O/c3_R$R.txt 2>&1 || { tail -20 $O/c3_R$R.txt; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_R$R.txt').read().strip().splitlines()[-1]); s=d['single']; print($R, d['R'], 'wall', s['wall_ms_min'], 'dp', s['dp_ms'], 'fin', s['finish_ms'], 'b2b', d['gcups'], 'bad', d['bad_status'])"
done
