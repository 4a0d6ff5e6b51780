#!/bin/bash
# Round 5: C3's single-alignment wall as the bench measures it (median of 5), twice.
set -o pipefail
out=gpurun_out/r05/${1:-c3single}
mkdir -p $out
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-h2h --no-affine --no-steady --configs C3 >> $out/bench.json 2>> $out/err.txt || exit 1
done
