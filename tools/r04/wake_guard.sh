# round 4: the s_wakeup build with the walk's op stores range-guarded (put_op): does the fault
# become BG_INTERNAL statuses?  Then the tree's metric for the guard's cost.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/wake; export TMPDIR=/tmp
cp biogarden_amd/libbiogarden_gpu.so /tmp/lib_tree.so
cp exp/wake.so biogarden_amd/libbiogarden_gpu.so
timeout -k 10 200 python3 bench.py --no-cpu --no-h2h --no-affine --configs "" --R 8 --waves 16 --pipeline 1 \
  > gpurun_out/r04/wake/guard.json 2> gpurun_out/r04/wake/guard.err
rc=$?
cp /tmp/lib_tree.so biogarden_amd/libbiogarden_gpu.so
echo "wake+guard rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/r04/wake/guard.json')); print(d['value'], d['all_status_ok'])" 2>/dev/null)"
grep -v amdgpu.ids gpurun_out/r04/wake/guard.err | tail -3
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 bench.py --no-cpu --no-h2h --no-affine --configs "" > gpurun_out/r04/wake/tree_m.json 2> gpurun_out/r04/wake/tree_m.err || exit 2
echo "tree metric $(python3 -c "import json; d=json.load(open('gpurun_out/r04/wake/tree_m.json')); print(d['value'], d['all_status_ok'])")"
