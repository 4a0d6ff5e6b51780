# C3 A/B of alternative library builds (exp/lib_$v.so for v in $VARS) against the tree's
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
cp biogarden_amd/libbiogarden_gpu.so /tmp/lib_tree.so
run() {
  echo -n "$1 "
  timeout -k 10 200 python tools/configs.py C3 --steps ${STEPS:-8} 2> gpurun_out/c3ab_$1.err | cut -c1-190 || { tail -5 gpurun_out/c3ab_$1.err; return 1; }
}
run tree || exit 1
for v in $VARS; do cp exp/lib_$v.so biogarden_amd/libbiogarden_gpu.so; run $v || exit 1; done
cp /tmp/lib_tree.so biogarden_amd/libbiogarden_gpu.so; run tree2 || exit 1
