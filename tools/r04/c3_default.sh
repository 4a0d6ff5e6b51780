# round 4: split tests with the new defaults (two WIDE DP streams, automatic exit pass beside a
# lone DP), then C3 pipelined + single at pipeline 3
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/c3def; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -x -v -s --timeout 100 --timeout-method thread > gpurun_out/r04/c3def/t_split.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|diag" gpurun_out/r04/c3def/t_split.log | cut -c1-200 | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/configs.py C3 --steps 20 --single 7 --pipeline 3 > gpurun_out/r04/c3def/c3.txt 2>&1; rc=$?; tail -2 gpurun_out/r04/c3def/c3.txt; exit $rc
