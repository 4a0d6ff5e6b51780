#!/bin/bash
# Round 5: the self-service traceback tests alone (a hang at slots = 6 in grp5b), printing as
# they go, then the rest of test_gpu_configs.
set -o pipefail
out=gpurun_out/r05/${1:-selfserve}
mkdir -p $out
timeout -k 10 240 python -u -m pytest -x -v -s --timeout 100 --timeout-method thread tests/test_gpu_configs.py -k self_service > $out/selfserve.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_configs.py > $out/configs.txt 2>&1 || exit 2
