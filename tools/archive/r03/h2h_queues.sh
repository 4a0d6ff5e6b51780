set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for q in 4 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu --no-affine --configs "C3" --steps 20 > gpurun_out/h2h_q$q.json 2>/dev/null || { echo "q $q failed"; continue; }
  python3 -c "import json; d=json.load(open('gpurun_out/h2h_q$q.json')); h=d['host_to_host']; c=d['configs']['C3']; print('queues $q', d['value'], 'h2h', h['gcups'], h['host_ms_per_batch']['fetch_d2h'], 'C3', c['value'], c['dp_ms'])"
done
