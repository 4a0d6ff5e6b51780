#!/bin/bash
# Round 5: the host_to_host leg with torch loaded: Python's cyclic GC over torch's objects?
set -o pipefail
out=gpurun_out/r05/${1:-gc}
mkdir -p $out
timeout -k 10 300 python -u tools/r05/h2h_probe.py --handles 4 --torch > $out/p_torch.jsonl 2> $out/p_torch.err && \
timeout -k 10 300 python -u tools/r05/h2h_probe.py --handles 4 --torch --extra 1 > $out/p_torch_x1.jsonl 2> $out/p_torch_x1.err && \
timeout -k 10 300 python -u tools/r05/h2h_probe.py --handles 4 > $out/p_plain.jsonl 2> $out/p_plain.err
