#!/bin/bash
# Round 5: C4's pipelined step at pipeline depth 2, 3 and 4, alternated (its run-to-run spread).
set -o pipefail
out=gpurun_out/r05/${1:-c4depth}
mkdir -p $out
for rep in 1 2 3; do
  for d in 2 3 4; do
    timeout -k 10 120 python3 tools/configs.py C4 --steps 20 --pipeline $d >> $out/c4_d$d.txt 2>&1 || exit 1
  done
done
