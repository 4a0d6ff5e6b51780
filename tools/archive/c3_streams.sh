# C3 with the alternating traceback streams (default) against one stream (BG_ONE_FIN_STREAM),
# pipeline depth 2 and 3, 12 steps; then the WIDE / C3 GPU tests
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for one in 0 1; do
  for p in 2 3; do
    if [ $one = 1 ]; then export BG_ONE_FIN_STREAM=1; else unset BG_ONE_FIN_STREAM; fi
    timeout -k 10 200 python tools/configs.py C3 --steps 12 --pipeline $p 2>&1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('one_stream=$one pipe=$p', d['gcups'], d['ms_per_step'], d['dp_ms'], d['finish_ms'], d['R'], d['bad_status'])" || exit 1
  done
done
unset BG_ONE_FIN_STREAM
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "wide or C3 or stream or export" --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; exit $rc
