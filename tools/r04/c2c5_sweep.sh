# round 4: C2 / C5 geometry sweep (DP strip height R x waves W, finish workgroup waves / slots)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/sweep; export TMPDIR=/tmp
for cfg in C2 C5; do
  for rw in "0 0" "2 2" "2 4" "2 8" "4 2" "4 4" "4 8"; do
    set -- $rw
    timeout -k 10 200 python tools/configs.py $cfg --steps 12 --R $1 --waves $2 > gpurun_out/r04/sweep/${cfg}_R$1_W$2.txt 2>&1 || { echo "$cfg R $1 W $2 failed"; tail -3 gpurun_out/r04/sweep/${cfg}_R$1_W$2.txt; continue; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/r04/sweep/${cfg}_R$1_W$2.txt').read().strip().splitlines()[-1]); print('$cfg R $1 W $2 ->', d['R'], d['waves'], d['gcups'], d['dp_ms'], d['finish_ms'])"
  done
  for fw in "1 2" "1 3" "2 3" "2 5" "4 5"; do
    set -- $fw
    BG_FIN_WAVES=$1 BG_FIN_SLOTS=$2 timeout -k 10 200 python tools/configs.py $cfg --steps 12 > gpurun_out/r04/sweep/${cfg}_fw$1_$2.txt 2>&1 || { echo "$cfg fin $1/$2 failed"; continue; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r04/sweep/${cfg}_fw$1_$2.txt').read().strip().splitlines()[-1]); print('$cfg fin waves $1 slots $2 ->', d['gcups'], d['dp_ms'], d['finish_ms'])"
  done
done
