# C3 over strip heights for the tree's library, then the same for exp/$ALT (if set)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
sweep() {
  for RR in ${RS:-2 3 4 5 8 10}; do
    timeout -k 10 200 python tools/configs.py C3 --steps 2 --R $RR 2>&1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1 R=$RR', d['gcups'], d['ms_per_step'], d['dp_ms'], d['finish_ms'], d['R'], d['waves'])" || return 1
  done
}
sweep tree || exit 1
[ -n "$ALT" ] || exit 0
cp exp/$ALT biogarden_amd/libbiogarden_gpu.so
sweep $ALT || exit 1
