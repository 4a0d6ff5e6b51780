#!/bin/bash
# Round 5: C4 bench line at one / two finish waves, alternated (noise check), with rocm-smi.
set -o pipefail
out=gpurun_out/r05/${1:-grp3}
mkdir -p $out
rocm-smi --showclocks --showpower --showtemp > $out/smi0.txt 2>&1
for fw in 1 2 1 2; do
  BG_FIN_WAVES=$fw timeout -k 10 200 python3 bench.py --no-cpu --no-h2h --no-affine --configs C4 >> $out/c4_w$fw.jsonl 2>> $out/c4.err || exit 3
done
rocm-smi --showclocks --showpower --showtemp > $out/smi1.txt 2>&1
