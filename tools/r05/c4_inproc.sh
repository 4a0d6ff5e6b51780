#!/bin/bash
# Round 5: C4's spread within one process: one handle prepares and times C4 four times in a row
# (200 steps each); three processes.
set -o pipefail
out=gpurun_out/r05/${1:-c4inproc}
mkdir -p $out
for rep in 1 2 3; do
  echo "== process $rep" >> $out/c4.txt
  timeout -k 10 150 python3 tools/configs.py C4 C4 C4 C4 --steps 200 --pipeline 3 >> $out/c4.txt 2>&1 || exit 1
done
