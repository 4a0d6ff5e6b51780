#!/bin/bash
# Round 5: the linear traceback's speculative recomputation (BG_SPEC="depth,rows"): M's value,
# DP / traceback times, and chunks recomputed per pair (tools/finish_timing.py, pipeline 1).
set -o pipefail
out=gpurun_out/r05/${1:-spec}
mkdir -p $out
for v in "2,128" "1,128" "1,64" "0,0" "2,128"; do
  t=$(echo $v | tr ',' '_')
  BG_SPEC=$v timeout -k 10 200 python3 bench.py --no-cpu --no-h2h --no-affine --configs "" > $out/m_$t.json 2> $out/m_$t.err || exit 1
  BG_SPEC=$v timeout -k 10 120 python3 tools/finish_timing.py 256 1 > $out/ft_$t.txt 2>&1 || exit 2
done
