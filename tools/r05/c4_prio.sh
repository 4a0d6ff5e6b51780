#!/bin/bash
# Round 5: C4 with the grouped DP at priority 1 (BG_DP_PRIO=1) against 0, alternated, pipeline 3,
# 20 steps each.
set -o pipefail
out=gpurun_out/r05/${1:-c4prio}
mkdir -p $out
run() { timeout -k 10 120 python3 tools/configs.py C4 --steps 20 --pipeline 3; }
for x in 0 1 0 1 0 1; do
  if [ $x = 1 ]; then BG_DP_PRIO=1 run >> $out/p1.txt 2>&1 || exit 1; else run >> $out/p0.txt 2>&1 || exit 2; fi
done
