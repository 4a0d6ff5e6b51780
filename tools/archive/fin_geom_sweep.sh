# finish workgroup shape for many-pair batches (BG_FIN_WAVES / BG_FIN_SLOTS) on C2 / C5
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for g in ${GEOMS:-0,0 2,0 2,4 4,0}; do
  IFS=, read -r FW FS <<< "$g"
  env $( [ $FW != 0 ] && echo BG_FIN_WAVES=$FW ) $( [ $FS != 0 ] && echo BG_FIN_SLOTS=$FS ) BG_DUMMY=1 \
    timeout -k 10 300 python tools/configs.py ${CFGS:-C2 C5} 2>&1 | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print('$g', d['config'], d['gcups'], d['ms_per_step'], d['dp_ms'], d['finish_ms'])" || exit 1
done
