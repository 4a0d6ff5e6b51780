# Round 6: the affine configurations' geometry and traceback shape re-checked with the options API
# (tools/configs.py, 12 pipelined steps): C5 and C2 over R x W x traceback waves / slots.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-r06/aff_sweep}; mkdir -p $O; export TMPDIR=/tmp
one() {  # config R W options tag
  BG_OPTIONS="$4" timeout -k 10 120 python3 tools/configs.py $1 --R $2 --waves $3 --steps 12 > $O/$5.json 2> $O/$5.err || { tail -3 $O/$5.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$5.json').read().strip().splitlines()[-1]); print('$5', d['gcups'], d['ms_per_step'], 'R', d['R'], 'W', d['waves'], 'dp', d['dp_ms'], 'fin', d['finish_ms'], 'bad', d['bad_status'])"
}
for cfg in C5 C2; do
  one $cfg 0 0 "" ${cfg}_auto || exit 1
  for R in 2 3 4; do
    for W in 2 4; do
      for fo in "" "fin_waves=2,fin_slots=3" "fin_waves=1,fin_slots=2" "fin_waves=4"; do
        tag=${cfg}_R${R}_W${W}_$(echo "${fo:-auto}" | tr ',=' '__')
        one $cfg $R $W "$fo" $tag || exit 1
      done
    done
  done
done
