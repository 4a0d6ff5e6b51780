#!/bin/bash
# Round 5: what slows the bench's host_to_host leg against the standalone probe.
set -o pipefail
out=gpurun_out/r05/${1:-ctx}
mkdir -p $out
timeout -k 10 300 python -u tools/r05/h2h_probe.py --handles 4 --torch > $out/p_torch.jsonl 2> $out/p_torch.err && \
timeout -k 10 300 python -u tools/r05/h2h_probe.py --handles 4 --extra 1 --c3 > $out/p_c3.jsonl 2> $out/p_c3.err && \
timeout -k 10 300 python -u tools/r05/h2h_probe.py --handles 4 --extra 1 --c3 --torch > $out/p_c3_torch.jsonl 2> $out/p_c3_torch.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --configs "" > $out/bench_noconf.json 2> $out/bench_noconf.err && \
timeout -k 10 300 python -u bench.py --group --group-devices 0 --steps 6 --warmup 2 > $out/group1.json 2> $out/group1.err
