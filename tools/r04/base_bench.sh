# round 4: default bench on a fresh box (the environment's GPU_MAX_HW_QUEUES kept)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04; export TMPDIR=/tmp
echo "env GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
timeout -k 10 600 python bench.py > gpurun_out/r04/base_bench.json 2> gpurun_out/r04/base_bench.err || { tail -20 gpurun_out/r04/base_bench.err; exit 1; }
python3 tools/summ_bench.py gpurun_out/r04/base_bench.json
