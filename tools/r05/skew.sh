#!/bin/bash
# Round 5: grouped DP with rows skewed in the lane — parity tests, C4 config test, C4 alone
# (finish timing, pipeline 1) and the C4 bench line.
set -o pipefail
out=gpurun_out/r05/${1:-skew}
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_grouped.py > $out/tests_grouped.txt 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_configs.py -k C4 > $out/tests_c4.txt 2>&1 || exit 2
BG_FINISH_TIMING=1 timeout -k 10 150 python tools/configs.py C4 --steps 2 --pipeline 1 > $out/c4_ft.txt 2>&1 || exit 3
for x in 1 2; do timeout -k 10 120 python3 tools/configs.py C4 --steps 20 --pipeline 3 >> $out/c4_p3.txt 2>&1 || exit 4; done
