#!/bin/bash
# Round 5: P = 8 against P = 4 on a batch twice C4's share (16 384 reads: rank 0 of 4), alone and
# pipelined, and the default planner's choice on C4 itself.
set -o pipefail
out=gpurun_out/r05/${1:-grp16b}
mkdir -p $out
for p in 8 4; do
  BG_GRP_P=$p timeout -k 10 150 python tools/configs.py C4 --world 4 --steps 2 --pipeline 1 > $out/c4w4_ft_p$p.txt 2>&1 || exit 3
  BG_GRP_P=$p timeout -k 10 150 python3 tools/configs.py C4 --world 4 --steps 20 --pipeline 3 > $out/c4w4_p3_p$p.txt 2>&1 || exit 4
done
timeout -k 10 150 python3 tools/configs.py C4 --steps 20 --pipeline 3 > $out/c4_default.txt 2>&1 || exit 5
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_configs.py -k C4 > $out/tests_c4.txt 2>&1 || exit 6
