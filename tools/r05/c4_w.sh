#!/bin/bash
# Round 5: C4's pipelined spread against the grouped DP's waves per workgroup (BG_GRP_W 1, 4, 8),
# three repetitions each, interleaved.
set -o pipefail
out=gpurun_out/r05/${1:-c4w}
mkdir -p $out
for rep in 1 2 3; do
  for w in 1 4 8; do
    BG_GRP_W=$w timeout -k 10 120 python3 tools/configs.py C4 --steps 20 --pipeline 3 >> $out/c4_w$w.txt 2>&1 || exit 1
  done
done
