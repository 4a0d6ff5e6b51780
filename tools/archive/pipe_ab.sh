# metric bench at pipeline depths 1-3 (DP and finish kernel times with and without overlap)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for p in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu --no-h2h --pipeline $p ${BENCH_ARGS} 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('pipeline $p', d['value'], d['ms_per_step'], r['kernel_ms'], r['finish_ms'])" || exit 1
done
