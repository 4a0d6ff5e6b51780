# Round 6: the export / group tests, then the group bench's kernel trace and plain run (after the
# compact scan became one wave).
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r06/${1:-gcheck2}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_export.py tests/test_gpu_group.py tests/test_gpu_stream.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/r06/group_trace.sh ${1:-gcheck2}/trace
