# A/B of the linear checkpoint traceback (asynchronous recompute default vs BG_FIN_SYNC=1 barriers): finish-kernel cycle breakdown
# on the metric pairs alone, then the bench and C3 / C4
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in 0 1; do
  if [ $v = 1 ]; then export BG_FIN_SYNC=1; fi
  echo "== BG_FIN_SYNC=$v"
  timeout -k 10 200 python tools/finish_timing.py 64 2>&1 | tail -2 || exit 1
  timeout -k 10 200 python bench.py --no-cpu --no-h2h 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('bench', d['value'], d['ms_per_step'], r['kernel_ms'], r['finish_ms'])" || exit 1
  timeout -k 10 300 python tools/configs.py C3 C4 2>&1 | tail -2 || exit 1
done
