#!/bin/bash
# Round 5: shared-stream rotation + split arena tests, then the default bench (host_to_host at the
# box's own GPU_MAX_HW_QUEUES).
set -o pipefail
out=gpurun_out/r05/${1:-s1}
mkdir -p $out
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}" > $out/env.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_stream.py tests/test_gpu_split.py > $out/tests.txt 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
