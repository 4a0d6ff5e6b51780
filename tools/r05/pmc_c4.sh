#!/bin/bash
# Round 5: C4's grouped DP and finish — instruction mix, wait and busy cycles, LDS (three passes,
# pipeline 1), BG_GRP_P as set by the caller.
set -o pipefail
out=gpurun_out/r05/${1:-pmcc4}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VMEM --output-format csv -d $out/p1 -o c4 -- \
  python3 tools/configs.py C4 --steps 2 --pipeline 1 > $out/p1.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $out/p2 -o c4 -- \
  python3 tools/configs.py C4 --steps 2 --pipeline 1 > $out/p2.txt 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --output-format csv -d $out/p3 -o c4 -- \
  python3 tools/configs.py C4 --steps 2 --pipeline 1 > $out/p3.txt 2>&1 || exit 3
python3 tools/pmc_summary.py $out > $out/summary_print.txt 2>&1
