#!/bin/bash
# Round 5: M's kernels' instruction mix (DP vs traceback) and the traceback's per-pair phases.
set -o pipefail
out=gpurun_out/r05/${1:-pmcm}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VMEM --output-format csv -d $out/p1 -o m -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu --no-h2h --no-affine --configs "" > $out/p1.json 2> $out/p1.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d $out/p2 -o m -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu --no-h2h --no-affine --configs "" > $out/p2.json 2> $out/p2.err || exit 2
timeout -k 10 120 python3 tools/finish_timing.py 256 1 > $out/fin_timing.txt 2>&1
