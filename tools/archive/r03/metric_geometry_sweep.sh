set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for rw in "8 16" "10 16" "8 10" "8 12" "5 16" "4 16" "10 12" "3 16"; do
  set -- $rw
  timeout -k 10 200 python bench.py --no-cpu --no-h2h --no-affine --configs "" --R $1 --waves $2 > gpurun_out/m_R$1_W$2.json 2>/dev/null || { echo "R $1 W $2 failed"; continue; }
  python3 -c "import json; d=json.load(open('gpurun_out/m_R$1_W$2.json')); r=d['roofline']; print('R $1 W $2', d['value'], d['ms_per_step'], r.get('kernel_ms'), r.get('finish_ms'))"
done
for p in 3 4; do
  timeout -k 10 200 python bench.py --no-cpu --no-h2h --no-affine --configs "" --pipeline $p > gpurun_out/m_p$p.json 2>/dev/null || exit 3
  python3 -c "import json; d=json.load(open('gpurun_out/m_p$p.json')); print('pipeline $p', d['value'], d['ms_per_step'])"
done
