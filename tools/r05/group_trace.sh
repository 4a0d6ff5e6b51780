#!/bin/bash
# Round 5: kernel trace of the pipelined group bench (one member): where the device idles.
set -o pipefail
out=gpurun_out/r05/${1:-gtrace}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/kt -o g -- python3 bench.py --group --gpus 1 --steps 10 --warmup 2 > $out/group1.json 2> $out/err.txt || exit 1
