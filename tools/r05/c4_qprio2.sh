#!/bin/bash
# Round 5: C4, DP streams at high queue priority (BG_QPRIO=1) against the default, six
# repetitions interleaved, and with four traceback slots (BG_FIN_SLOTS=4, 18 KB of LDS per
# traceback workgroup instead of 23 KB).
set -o pipefail
out=gpurun_out/r05/${1:-c4q2}
mkdir -p $out
for rep in 1 2 3 4 5 6; do
  BG_QPRIO=0 timeout -k 10 120 python3 tools/configs.py C4 --steps 20 --pipeline 3 >> $out/c4_q0.txt 2>&1 || exit 1
  BG_QPRIO=1 timeout -k 10 120 python3 tools/configs.py C4 --steps 20 --pipeline 3 >> $out/c4_q1.txt 2>&1 || exit 2
  BG_QPRIO=1 BG_FIN_SLOTS=4 timeout -k 10 120 python3 tools/configs.py C4 --steps 20 --pipeline 3 >> $out/c4_q1s4.txt 2>&1 || exit 3
done
