#!/bin/bash
# Round 5: MA's round-4 drop: the walker's priority (BG_FIN_PRIO=1 restores priority 3 for
# many-pair batches) A/B, interleaved, with C2 and C5 beside.
set -o pipefail
out=gpurun_out/r05/${1:-prio}
mkdir -p $out
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-h2h --configs C2,C5 > $out/def_$r.json 2> $out/def_$r.err || exit 1
  BG_FIN_PRIO=1 timeout -k 10 300 python -u bench.py --no-cpu --no-h2h --configs C2,C5 > $out/prio_$r.json 2> $out/prio_$r.err || exit 1
done
