# A/B of library builds on the GPU box: the tree's libbiogarden_gpu.so against variants/<name>.so, in
# two interleaved passes (drift control).  usage: LIBS="a b" WHAT="M C3 C2" bash tools/ab.sh
#   M   bench.py metric leg only (no CPU / h2h / affine / configs legs)
#   MA  bench.py's affine leg's workload as the headline (--open -11 --extend -1)
#   Cn  tools/configs.py Cn --steps 12
#   G   bench.py --group (one member, three batches in flight, host to host)
# ENV_<name> (e.g. ENV_tree="BG_WIDE_W=8") sets environment for one variant.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
cp biogarden_amd/libbiogarden_gpu.so /tmp/lib_tree.so
run_one() {   # $1 variant, $2 what
  local envv; envv=$(eval echo \${ENV_$1})
  case $2 in
    M)  env $envv timeout -k 10 200 python bench.py --no-cpu --no-h2h --no-affine --configs "" 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$1 M', d['value'], d['ms_per_step'], r['kernel_ms'], r['finish_ms'])" ;;
    MA) env $envv timeout -k 10 200 python bench.py --no-cpu --no-h2h --no-affine --configs "" --open -11 --extend -1 --steps 10 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$1 MA', d['value'], d['ms_per_step'], r['kernel_ms'], r['finish_ms'])" ;;
    G)  env $envv timeout -k 10 300 python bench.py --group --gpus 1 --steps 20 --warmup 3 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 G', d['value'], d['ms_per_step'], d['host_ms_per_step'])" ;;
    C*) env $envv timeout -k 10 200 python tools/configs.py $2 --steps 12 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1 $2', d['gcups'], d['ms_per_step'], d['dp_ms'], d['finish_ms'], 'R', d['R'], 'W', d['waves'])" ;;
  esac
}
for pass in 1 2; do
  for v in tree $LIBS; do
    if [ $v = tree ]; then cp /tmp/lib_tree.so biogarden_amd/libbiogarden_gpu.so; else cp variants/$v.so biogarden_amd/libbiogarden_gpu.so; fi
    for w in ${WHAT:-M C3}; do run_one $v $w || { cp /tmp/lib_tree.so biogarden_amd/libbiogarden_gpu.so; exit 1; }; done
  done
done
cp /tmp/lib_tree.so biogarden_amd/libbiogarden_gpu.so
