# round 4: DP workgroups per CU capped by padded LDS (BG_DP_CAP) so tracebacks run beside them
# (the BG_DP_CAP knob was removed after this experiment: profiles/r04/geometry/dp_cap_lds_padding.txt)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/dpcap; export TMPDIR=/tmp
for cfg in "C5 4 2 0" "C5 4 2 8" "C5 4 2 6" "C5 4 2 4" "C5 2 2 8" "C5 2 2 6" "C2 2 4 6" "C2 2 4 4" "C4 3 1 24" "C4 3 1 16"; do set -- $cfg
  BG_DP_CAP=$4 timeout -k 10 200 python tools/configs.py $1 --steps 20 --R $2 --waves $3 > gpurun_out/r04/dpcap/cfg.txt 2>&1 || { tail -5 gpurun_out/r04/dpcap/cfg.txt; exit 4; }
  echo "[$cfg] $(python3 -c "
import json
for l in open('gpurun_out/r04/dpcap/cfg.txt'):
    if l.startswith('{'): d=json.loads(l); print(d['config'], d['gcups'], 'dp', d['dp_ms'], 'fin', d['finish_ms'], 'bad', d['bad_status'], end=' | ')
")"
done
