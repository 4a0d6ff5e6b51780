# round 4: the whole GPU test suite (split tests and the full-size C3 string test included), then
# the finish-kernel phase breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04/suite; export TMPDIR=/tmp
grep MemAvailable /proc/meminfo
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04/suite/t_gpu.log 2>&1; rc=$?
grep -cE "PASSED" gpurun_out/r04/suite/t_gpu.log; grep -E "FAIL|Error|SKIP|passed|failed" gpurun_out/r04/suite/t_gpu.log | cut -c1-200 | tail -15; [ $rc -eq 0 ] || exit $rc
bash tools/r04/fin_phases.sh
