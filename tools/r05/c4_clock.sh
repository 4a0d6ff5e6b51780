#!/bin/bash
# Round 5: C4's run-to-run spread against the GPU's clock, power and temperature: rocm-smi
# sampled in the background (read-only) while six C4 runs and two metric runs go, each run's
# start / end time logged.
set -o pipefail
out=gpurun_out/r05/${1:-c4clk}
mkdir -p $out
( while true; do echo "T $(date +%s.%N)"; timeout 5 rocm-smi --showclocks --showpower --showtemp 2>&1 | grep -E "sclk|mclk|Power|Temperature|fclk"; sleep 0.3; done ) > $out/smi.txt &
smi=$!
for rep in 1 2 3 4 5 6; do
  echo "start c4 $rep $(date +%s.%N)" >> $out/runs.txt
  timeout -k 10 120 python3 tools/configs.py C4 --steps 20 --pipeline 3 >> $out/c4.txt 2>&1 || { kill $smi; exit 1; }
  echo "end c4 $rep $(date +%s.%N)" >> $out/runs.txt
done
for rep in 1 2; do
  echo "start m $rep $(date +%s.%N)" >> $out/runs.txt
  timeout -k 10 120 python3 bench.py --no-cpu --no-h2h --no-affine --configs "" >> $out/m.json 2>> $out/err.txt || { kill $smi; exit 2; }
  echo "end m $rep $(date +%s.%N)" >> $out/runs.txt
done
kill $smi
