#!/bin/bash
# Round 5: grouped DP with the last-row key folded in the DP — parity tests, C4 config test, C4
# bench line at one / two finish waves, and the finish timing.
set -o pipefail
out=gpurun_out/r05/${1:-grp2}
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_grouped.py tests/test_gpu_lastrow.py > $out/tests_grouped.txt 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_configs.py -k C4 > $out/tests_c4.txt 2>&1 || exit 2
for fw in 1 2; do
  BG_FIN_WAVES=$fw timeout -k 10 200 python3 bench.py --no-cpu --no-h2h --no-affine --configs C4 > $out/c4_w$fw.json 2> $out/c4_w$fw.err || exit 3
  BG_FIN_WAVES=$fw BG_FINISH_TIMING=1 timeout -k 10 150 python tools/configs.py C4 --steps 2 --pipeline 1 > $out/c4_ft_w$fw.txt 2>&1 || exit 4
done
