#!/bin/bash
# Round 5: C4's steady state (200 steps) in a lone process, after torch's GPU init, and as the
# bench's config leg (after the metric's legs, same handle); twice each, interleaved.
set -o pipefail
out=gpurun_out/r05/${1:-c4ctx}
mkdir -p $out
for rep in 1 2; do
  timeout -k 10 120 python3 tools/configs.py C4 --steps 200 --pipeline 3 >> $out/lone.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/configs.py C4 --steps 200 --pipeline 3 --torch-init >> $out/torch.txt 2>&1 || exit 2
  timeout -k 10 200 python3 bench.py --no-cpu --no-h2h --no-affine --configs C4 >> $out/bench.json 2>> $out/err.txt || exit 3
done
