# planner variants: C2 / C5 with the tree's library and each exp/lib_*.so
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
cp biogarden_amd/libbiogarden_gpu.so /tmp/lib_tree.so
for L in /tmp/lib_tree.so exp/lib_*.so; do
  cp $L biogarden_amd/libbiogarden_gpu.so
  echo "== $L"
  timeout -k 10 300 python tools/configs.py C2 C5 2>&1 | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print(d['config'], d['gcups'], d['ms_per_step'], d['dp_ms'], d['finish_ms'], 'R', d['R'], 'W', d['waves'])" || exit 1
done
cp /tmp/lib_tree.so biogarden_amd/libbiogarden_gpu.so
