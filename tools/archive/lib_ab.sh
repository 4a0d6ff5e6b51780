# A/B of an alternative build of the library (exp/$ALT) against the tree's: finish breakdown + bench
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() {
  timeout -k 10 200 python tools/finish_timing.py 64 2>&1 | tail -2 || return 1
  timeout -k 10 200 python bench.py --no-cpu --no-h2h 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('bench', d['value'], d['ms_per_step'], r['kernel_ms'], r['finish_ms'])"
}
echo "== tree"; run || exit 1
cp exp/$ALT biogarden_amd/libbiogarden_gpu.so
echo "== $ALT"; run || exit 1
