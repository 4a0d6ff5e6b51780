# Round 6: kernel trace of the pipelined group bench (one member) beside the handle's
# host-to-host leg: the gaps between DPs and what runs in them (tools/r05/trace_gaps.py).
set -o pipefail
out=gpurun_out/r06/${1:-gtrace}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/kt -o g -- python3 bench.py --group --gpus 1 --steps 10 --warmup 2 > $out/group1.json 2> $out/err.txt || exit 1
python3 tools/r05/trace_gaps.py $out/kt > $out/gaps.txt && cat $out/gaps.txt
timeout -k 10 300 python3 bench.py --group --gpus 1 --steps 20 --warmup 3 > $out/group1_plain.json 2> $out/err2.txt || exit 2
tail -1 $out/group1_plain.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('group', d['value'], d['ms_per_step'], d['host_ms_per_step'])"
