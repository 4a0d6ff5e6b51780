# Round 6: (1) C4's step spread across processes (round 5: 7 153 - 9 643 GCUPS), eight 20-step
# and four 200-step processes; (2) bench.py --group at 1 and 2 virtual members (the expansion now
# one pool pass over all members); (3) the SPAN geometry sweep (tools/r06/span_sweep.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-r06/misc1}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2 3 4 5 6 7 8; do
  timeout -k 10 120 python3 tools/configs.py C4 --steps 20 --pipeline 3 >> $O/c4_s20.txt 2>&1 || exit 1
done
for rep in 1 2 3 4; do
  timeout -k 10 120 python3 tools/configs.py C4 --steps 200 --pipeline 3 >> $O/c4_s200.txt 2>&1 || exit 2
done
grep -h "GCUPS\|gcups" $O/c4_s20.txt $O/c4_s200.txt | head -20
for devs in 0 0,0; do
  timeout -k 10 240 python3 bench.py --group --group-devices $devs --steps 20 --warmup 3 > $O/group_$devs.json 2> $O/group_$devs.err || { tail -5 $O/group_$devs.err; exit 3; }
  python3 -c "import json; d=json.load(open('$O/group_$devs.json')); print('$devs', d['value'], d['ms_per_step'], d['host_ms_per_step'], d['all_status_ok'])"
done
bash tools/r06/span_sweep.sh ${1:-r06/misc1}/sweep
