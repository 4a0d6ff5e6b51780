# Many-pair batches with one traceback stream (default) against two alternating ones
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for two in 0 1; do
  if [ $two = 1 ]; then export BG_TWO_FIN_STREAMS=1; else unset BG_TWO_FIN_STREAMS; fi
  timeout -k 10 400 python tools/configs.py C2 C4 C5 2>&1 | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print('two=$two', d['config'], d['gcups'], d['ms_per_step'], d['dp_ms'], d['finish_ms'])" || exit 1
  timeout -k 10 200 python bench.py --no-cpu --no-h2h 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; a=d['affine']; print('two=$two M', d['value'], d['ms_per_step'], r['kernel_ms'], r['finish_ms'], 'MA', a['value'])" || exit 1
done
