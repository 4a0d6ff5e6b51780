#!/bin/bash
# Round 5: M's geometry re-checked after the round's DP changes (repeat-row-n1 last strip):
# R x W sweep of the metric, default first and last.
set -o pipefail
out=gpurun_out/r05/${1:-mgeom}
mkdir -p $out
run() { timeout -k 10 120 python3 bench.py --no-cpu --no-h2h --no-affine --configs "" "$@"; }
run > $out/default_a.json 2> $out/err.txt || exit 1
for rw in "10 16" "10 12" "8 12" "8 20" "5 16" "10 20"; do
  set -- $rw
  run --R $1 --waves $2 > $out/r$1_w$2.json 2>> $out/err.txt || exit 2
done
run > $out/default_b.json 2>> $out/err.txt || exit 3
