# Round 6: the pipelined group (one member) beside the handle on one box, then the group at three
# host pool sizes (BG_HOST_THREADS): is the collect's expansion bound by the pool's threads?
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r06/${1:-gthr}; mkdir -p $O; export TMPDIR=/tmp
bash tools/r06/group_rep.sh ${1:-gthr} || exit 1
for t in 8 32 4; do
  BG_HOST_THREADS=$t timeout -k 10 300 python3 bench.py --group --gpus 1 --steps 20 --warmup 3 > $O/group_t$t.json 2> $O/group_t$t.err || { tail -5 $O/group_t$t.err; exit 2; }
  tail -1 $O/group_t$t.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('threads $t group', d['value'], d['ms_per_step'], d['host_ms_per_step'])"
done
