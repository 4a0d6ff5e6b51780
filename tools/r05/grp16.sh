#!/bin/bash
# Round 5: eight pairs per wave in 16-bit halves (bg_grp16_kernel.hip) — parity, then C4 alone
# and pipelined at P = 8 and 4.
set -o pipefail
out=gpurun_out/r05/${1:-grp16}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_grouped.py > $out/tests_grouped.txt 2>&1 || exit 1
for p in 8 4; do
  BG_GRP_P=$p BG_FINISH_TIMING=1 timeout -k 10 150 python tools/configs.py C4 --steps 2 --pipeline 1 > $out/c4_ft_p$p.txt 2>&1 || exit 3
done
for p in 8 4 8 4; do
  BG_GRP_P=$p timeout -k 10 120 python3 tools/configs.py C4 --steps 20 --pipeline 3 >> $out/c4_p3_p$p.txt 2>&1 || exit 4
done
