# A/B of alternative library builds (exp/lib_$v.so for v in $VARS) against the tree's: bench
# (metric + affine leg) for each, then the tree again.  Prints value / step / DP / finish ms.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
cp biogarden_amd/libbiogarden_gpu.so /tmp/lib_tree.so
run() {
  timeout -k 10 240 python bench.py --no-cpu --no-h2h --steps 20 --warmup 5 2> gpurun_out/ab_$1.err > gpurun_out/ab_$1.json || { tail -5 gpurun_out/ab_$1.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$1.json')); r=d['roofline']; a=d['affine']; print('$1', d['value'], d['ms_per_step'], r['kernel_ms'], r['finish_ms'], 'MA', a['value'], a['ms_per_step'], a['roofline']['kernel_ms'], a['roofline']['finish_ms'])"
}
run tree || exit 1
for v in $VARS; do cp exp/lib_$v.so biogarden_amd/libbiogarden_gpu.so; run $v || exit 1; done
cp /tmp/lib_tree.so biogarden_amd/libbiogarden_gpu.so; run tree2 || exit 1
