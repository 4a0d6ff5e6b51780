# Round 6: the pipelined group (one member) three times beside the handle's own legs on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r06/${1:-grep}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --no-cpu --configs '' --no-affine --no-steady > $O/handle.json 2> $O/handle.err || { tail -5 $O/handle.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/handle.json')); print('handle', d['value'], 'h2h', d['host_to_host']['gcups'])"
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --group --gpus 1 --steps 20 --warmup 3 > $O/group_$r.json 2> $O/group_$r.err || { tail -5 $O/group_$r.err; exit 2; }
  tail -1 $O/group_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('group', d['value'], d['ms_per_step'], d['host_ms_per_step'])"
done
