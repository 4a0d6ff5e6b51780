#!/bin/bash
# Round 5: C4's pipelined DP against HIP stream (queue) priority (BG_QPRIO: 1 DP streams high,
# 2 traceback streams low, 3 both), three repetitions, interleaved; then the metric at 0 / 1.
set -o pipefail
out=gpurun_out/r05/${1:-c4q}
mkdir -p $out
for rep in 1 2 3; do
  for q in 0 1 2 3; do
    BG_QPRIO=$q timeout -k 10 120 python3 tools/configs.py C4 --steps 20 --pipeline 3 >> $out/c4_q$q.txt 2>&1 || exit 1
  done
done
for q in 0 1 0 1; do
  BG_QPRIO=$q timeout -k 10 120 python3 bench.py --no-cpu --no-h2h --no-affine --configs "" >> $out/m_q$q.json 2>> $out/err.txt || exit 2
done
