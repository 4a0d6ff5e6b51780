#!/bin/bash
# Round 5: M's traceback workgroup re-checked (walker + helper waves, chunk slots), two
# interleaved rounds; the default first.
set -o pipefail
out=gpurun_out/r05/${1:-mfin}
mkdir -p $out
run() { timeout -k 10 120 python3 bench.py --no-cpu --no-h2h --no-affine --configs "" > $out/$1.json 2>> $out/err.txt; }
for r in a b; do
  run def_$r || exit 1
  BG_FIN_WAVES=3 run w3_$r || exit 2
  BG_FIN_WAVES=2 BG_FIN_SLOTS=5 run w2s5_$r || exit 3
  BG_FIN_WAVES=4 BG_FIN_SLOTS=6 run w4s6_$r || exit 4
done
