#!/bin/bash
# Round 5: the last-row tests, the whole GPU suite, smoke, then the default bench (stop at the
# first failure).
set -o pipefail
out=gpurun_out/r05/${1:-full}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lastrow.py > $out/tests_lastrow.txt 2>&1 || exit 1
timeout -k 10 1500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $out/gpu_tests.txt 2>&1 || exit 2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit 3
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err
