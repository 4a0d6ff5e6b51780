# Round 6: the group's collect with asynchronous exports (one host wait per collect): the group
# tests, then bench.py --group at 1 and 2 virtual members, and the SPAN plan at 64 / 128 pairs.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-r06/group_check}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_group.py tests/test_gpu_span.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for devs in 0 0,0; do
  timeout -k 10 240 python3 bench.py --group --group-devices $devs --steps 20 --warmup 3 > $O/group_$devs.json 2> $O/group_$devs.err || { tail -5 $O/group_$devs.err; exit 3; }
  grep "^{" $O/group_$devs.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$devs', d['value'], d['ms_per_step'], d['host_ms_per_step'], d['all_status_ok'])"
done
for p in 128 64; do
  timeout -k 10 240 python bench.py --pairs $p --steps 20 --warmup 3 --no-cpu --configs '' --no-affine --no-h2h --no-steady > $O/p$p.json 2> $O/p$p.err || { tail -20 $O/p$p.err; exit 4; }
  python3 -c "import json; d=json.load(open('$O/p$p.json')); k=d['config']['kernel']; print($p, d['value'], d['ms_per_step'], 'R', k['R'], 'W', k['waves'], 'wide', k['wide'], 'dp', d['roofline']['dp_ms'], 'fin', d['roofline']['finish_ms'])"
done
