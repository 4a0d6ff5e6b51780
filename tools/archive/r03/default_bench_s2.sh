set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/final_s2; export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/final_s2/default_bench.json 2> gpurun_out/final_s2/default_bench.err || { tail -20 gpurun_out/final_s2/default_bench.err; exit 1; }
python3 tools/summ_bench.py gpurun_out/final_s2/default_bench.json
