#!/bin/bash
# Round 5: strings downloaded by a kernel into host-mapped memory (bg_io.hip) against the
# copy-engine form (BG_DL_COPY=1), with and without PyTorch's HIP runtime; then the stream tests
# and the default bench.
set -o pipefail
out=gpurun_out/r05/${1:-dl}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_stream.py > $out/tests_stream.txt 2>&1 && \
timeout -k 10 300 python -u tools/r05/h2h_probe.py --handles 4 --torch > $out/p_torch.jsonl 2> $out/p_torch.err && \
timeout -k 10 300 python -u tools/r05/h2h_probe.py --handles 4 > $out/p_plain.jsonl 2> $out/p_plain.err && \
BG_DL_COPY=1 timeout -k 10 300 python -u tools/r05/h2h_probe.py --handles 4 --torch > $out/p_torch_copy.jsonl 2> $out/p_torch_copy.err && \
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
