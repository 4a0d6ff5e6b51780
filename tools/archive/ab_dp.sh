# A/B of an alternative library build (exp/$ALT): DP timeline of pair 0 at R=8 W=16 (pipeline 1)
# and the bench (no CPU leg, no host-to-host leg), tree first
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() {
  BG_DP_TIMING=1 timeout -k 10 200 python tools/dp_timeline.py --R ${TL_R:-8} --waves ${TL_W:-16} > gpurun_out/tl_$1.txt 2>&1 || { tail -20 gpurun_out/tl_$1.txt; return 1; }
  grep -E "run 1|span" gpurun_out/tl_$1.txt | tail -2 | cut -c1-200
  timeout -k 10 200 python bench.py --no-cpu --no-h2h ${BENCH_ARGS} 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; a=d.get('affine') or {}; print('bench', d['value'], d['ms_per_step'], r['kernel_ms'], r['finish_ms'], 'affine', a.get('value'), a.get('roofline',{}).get('kernel_ms'))"
}
echo "== tree"; run tree || exit 1
cp exp/$ALT biogarden_amd/libbiogarden_gpu.so
echo "== $ALT"; run alt || exit 1
