set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for e in "X=1" "HSA_ENABLE_SDMA=0" "HIP_FORCE_QUEUE_PROFILING=0"; do
  env $e timeout -k 10 300 python bench.py --no-cpu --no-affine --configs "" --steps 10 > gpurun_out/h2h_env.json 2>/dev/null || { echo "$e failed"; continue; }
  python3 -c "import json; d=json.load(open('gpurun_out/h2h_env.json')); h=d['host_to_host']; print('$e', d['value'], h['gcups'], h['host_ms_per_batch'])"
done
