#!/bin/bash
# Round 5: 16-byte gap runs in the finish — C4 finish timing, then the whole GPU suite, then the
# default bench (stop at the first failure).
set -o pipefail
out=gpurun_out/r05/${1:-grp5}
mkdir -p $out
BG_FINISH_TIMING=1 timeout -k 10 150 python tools/configs.py C4 --steps 2 --pipeline 1 > $out/c4_ft.txt 2>&1 || exit 4
timeout -k 10 1500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $out/gpu_tests.txt 2>&1 || exit 2
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err
