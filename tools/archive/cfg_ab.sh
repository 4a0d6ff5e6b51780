# configs (C2 C4 C5 + metric + MA via bench) for the tree's library, then exp/$ALT; repeated REP times
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
cp biogarden_amd/libbiogarden_gpu.so gpurun_out/lib_tree.so
run() {
  timeout -k 10 300 python tools/configs.py ${CFGS:-C2 C4 C5} --steps 3 2>&1 | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print('$1', d['config'], d['gcups'], d['ms_per_step'], d['dp_ms'], d['finish_ms'])" || return 1
  timeout -k 10 200 python bench.py --no-cpu --no-h2h 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; a=d['affine']; print('$1 M', d['value'], d['ms_per_step'], r['kernel_ms'], r['finish_ms'], 'MA', a['value'], a['ms_per_step'], a['roofline']['kernel_ms'], a['roofline']['finish_ms'])" || return 1
}
for i in $(seq ${REP:-1}); do
  cp gpurun_out/lib_tree.so biogarden_amd/libbiogarden_gpu.so; run tree || exit 1
  cp exp/$ALT biogarden_amd/libbiogarden_gpu.so; run $ALT || exit 1
done
cp gpurun_out/lib_tree.so biogarden_amd/libbiogarden_gpu.so   # leave the tree's library in place
rm -f gpurun_out/lib_tree.so
