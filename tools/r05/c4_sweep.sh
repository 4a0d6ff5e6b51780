#!/bin/bash
# Round 5: C4 grouped geometry — DP waves per workgroup (BG_GRP_W) and traceback slots
# (BG_FIN_SLOTS), pipeline 3, 20 steps each; the default before and after.
set -o pipefail
out=gpurun_out/r05/${1:-c4sweep}
mkdir -p $out
run() { timeout -k 10 120 python3 tools/configs.py C4 --steps 20 --pipeline 3; }
run > $out/default_a.txt 2>&1 || exit 1
for w in 2 8 16; do BG_GRP_W=$w run > $out/w$w.txt 2>&1 || exit 2; done
for s in 4 8; do BG_FIN_SLOTS=$s run > $out/s$s.txt 2>&1 || exit 3; done
BG_FIN_WAVES=2 run > $out/fw2.txt 2>&1 || exit 4
run > $out/default_b.txt 2>&1 || exit 5
