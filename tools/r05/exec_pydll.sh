#!/bin/bash
set -o pipefail
out=gpurun_out/r05/${1:-pydll}
mkdir -p $out
H2H_PYDLL=1 timeout -k 10 300 python -u tools/r05/h2h_probe.py --handles 4 --torch > $out/p_torch_pydll.jsonl 2> $out/p_torch_pydll.err && \
timeout -k 10 300 python -u tools/r05/h2h_probe.py --handles 4 --torch > $out/p_torch.jsonl 2> $out/p_torch.err
