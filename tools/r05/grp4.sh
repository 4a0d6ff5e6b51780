#!/bin/bash
# Round 5: C4 bench line with the last-row key folded in the grouped DP or in the finish
# (BG_GRP_FOLD=0), alternated in one call.
set -o pipefail
out=gpurun_out/r05/${1:-grp4}
mkdir -p $out
for f in 1 0 1 0; do
  BG_GRP_FOLD=$f timeout -k 10 200 python3 bench.py --no-cpu --no-h2h --no-affine --configs C4 >> $out/c4_f$f.jsonl 2>> $out/c4.err || exit 3
done
for f in 1 0; do
  BG_GRP_FOLD=$f BG_FINISH_TIMING=1 timeout -k 10 150 python tools/configs.py C4 --steps 2 --pipeline 1 > $out/c4_ft_f$f.txt 2>&1 || exit 4
done
