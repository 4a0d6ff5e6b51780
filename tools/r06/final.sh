# Round 6 final validation of the committed build: every GPU test, smoke(), the default bench
# (all legs, CPU baseline included).  usage: bash tools/r06/final.sh <out under gpurun_out>
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-r06/final}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 2; }
cat $O/smoke.txt | tail -1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
python3 tools/summ_bench.py $O/bench.json
