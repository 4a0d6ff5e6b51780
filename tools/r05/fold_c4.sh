#!/bin/bash
# Round 5: C4's traceback before the walk (end-cell folds with 8 loads in flight), pipeline 3 / 1,
# then the priority A/B of tools/r05/prio_ab.sh.
set -o pipefail
out=gpurun_out/r05/${1:-fold}
mkdir -p $out
for p in 3 1; do
  BG_FINISH_TIMING=1 timeout -k 10 150 python tools/configs.py C4 --steps 2 --pipeline $p > $out/c4_p$p.txt 2>&1 || exit 4
done
bash tools/r05/prio_ab.sh ${1:-fold}/prio
