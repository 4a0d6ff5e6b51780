#!/bin/bash
# Round 5: the metric at pipeline depth 2 / 3 / 4 (K = 20 value and the 200-step steady state),
# two interleaved rounds.
set -o pipefail
out=gpurun_out/r05/${1:-mdepth}
mkdir -p $out
for r in a b; do
  for d in 3 2 4; do
    timeout -k 10 120 python3 bench.py --no-cpu --no-h2h --no-affine --configs "" --pipeline $d > $out/d${d}_$r.json 2>> $out/err.txt || exit 1
  done
done
