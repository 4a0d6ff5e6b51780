#!/bin/bash
# Round 5: grouped DP at 4 and 2 pairs per wave — parity tests, the C4 config test, then C4's bench
# line and finish timing at BG_GRP_P=4 / 2, alternated.
set -o pipefail
out=gpurun_out/r05/${1:-grp6}
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_grouped.py > $out/tests_grouped.txt 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_configs.py -k C4 > $out/tests_c4.txt 2>&1 || exit 2
for p in 4 2 4 2; do
  BG_GRP_P=$p timeout -k 10 200 python3 bench.py --no-cpu --no-h2h --no-affine --configs C4 >> $out/c4_p$p.jsonl 2>> $out/c4.err || exit 3
done
for p in 4 2; do
  BG_GRP_P=$p BG_FINISH_TIMING=1 timeout -k 10 150 python tools/configs.py C4 --steps 2 --pipeline 1 > $out/c4_ft_p$p.txt 2>&1 || exit 4
done
