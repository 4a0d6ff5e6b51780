#!/bin/bash
# Round 5 first GPU pass on the restored tree: group, stream and split tests, then the default bench.
set -o pipefail
out=gpurun_out/r05/${1:-first}
mkdir -p $out
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}" > $out/env.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_group.py tests/test_gpu_stream.py tests/test_gpu_split.py > $out/tests.txt 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
