#!/bin/bash
# Round 5: host_to_host leg probes (per-call host timings; a kernel + copy timeline).
set -o pipefail
out=gpurun_out/r05/${1:-h2h}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/r05/h2h_probe.py --handles 2,3,4 --pipeline 2 --extra 0 > $out/probe_x0.jsonl 2> $out/probe_x0.err && \
timeout -k 10 300 python -u tools/r05/h2h_probe.py --handles 4 --pipeline 2,3 --extra 1 > $out/probe_x1.jsonl 2> $out/probe_x1.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $out/trace -o run -- \
  python -u tools/r05/h2h_probe.py --handles 4 --pipeline 2 --rounds 12 > $out/trace_probe.jsonl 2> $out/trace.err &&
timeout -k 10 300 python -u bench.py --group --group-devices 0 --steps 6 --warmup 2 > $out/group1.json 2> $out/group1.err && \
timeout -k 10 300 python -u bench.py --group --group-devices 0,0 --steps 6 --warmup 2 > $out/group2.json 2> $out/group2.err
