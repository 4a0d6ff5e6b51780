#!/bin/bash
# Round 5: grouped DP (bg_grp_kernel.hip) — its parity tests, the C4 config test, then C4's
# bench line grouped and one wave per pair (BG_GROUPED=0), and the finish timing of both.
set -o pipefail
out=gpurun_out/r05/${1:-grp}
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_grouped.py > $out/tests_grouped.txt 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_configs.py -k C4 > $out/tests_c4.txt 2>&1 || exit 2
for g in 1 0; do
  BG_GROUPED=$g timeout -k 10 200 python3 bench.py --no-cpu --no-h2h --no-affine --configs C4 > $out/c4_g$g.json 2> $out/c4_g$g.err || exit 3
  BG_GROUPED=$g BG_FINISH_TIMING=1 timeout -k 10 150 python tools/configs.py C4 --steps 2 --pipeline 1 > $out/c4_ft_g$g.txt 2>&1 || exit 4
done
