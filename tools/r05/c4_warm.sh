#!/bin/bash
# Round 5: is C4's spread the GPU clock ramping up inside a short timed region?  20 timed steps
# (26 ms) after 2 executes, after >= 300 ms of untimed executes, and 200 timed steps; six
# repetitions interleaved.
set -o pipefail
out=gpurun_out/r05/${1:-c4warm}
mkdir -p $out
for rep in 1 2 3 4 5 6; do
  timeout -k 10 120 python3 tools/configs.py C4 --steps 20 --pipeline 3 >> $out/s20.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/configs.py C4 --steps 20 --pipeline 3 --warm-ms 300 >> $out/s20_w300.txt 2>&1 || exit 2
  timeout -k 10 120 python3 tools/configs.py C4 --steps 200 --pipeline 3 >> $out/s200.txt 2>&1 || exit 3
done
