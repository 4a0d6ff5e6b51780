#!/bin/bash
# Round 5: multi-device group (virtual shards on device 0, RCCL self-send), shared-stream rotation,
# then the default bench.
set -o pipefail
out=gpurun_out/r05/${1:-g1}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_group.py tests/test_gpu_stream.py tests/test_gpu_export.py > $out/tests.txt 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --configs "" --no-cpu > $out/bench.json 2> $out/bench.err
