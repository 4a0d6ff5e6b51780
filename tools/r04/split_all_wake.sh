# round 4: every split test (bounded), then the plain wakeup variant at R = 8 / W = 16
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/conc2; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -x -v -s --timeout 100 --timeout-method thread > gpurun_out/r04/conc2/t_all.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|diag" gpurun_out/r04/conc2/t_all.log | cut -c1-220 | tail -30; [ $rc -eq 0 ] || exit $rc
bash tools/r04/wake_plain.sh
