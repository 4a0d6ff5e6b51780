# metric bench over strip height / wave count / pipeline depth: GCUPS, step, DP and finish ms
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for cfg in ${CFGS:-8,16,3 10,16,3 10,16,2 5,16,3 4,16,3}; do
  IFS=, read -r RR WW PP <<< "$cfg"
  timeout -k 10 200 python bench.py --no-cpu --no-h2h --no-affine --R $RR --waves $WW --pipeline $PP 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$cfg', d['value'], d['ms_per_step'], r['kernel_ms'], r['finish_ms'])" || exit 1
done
