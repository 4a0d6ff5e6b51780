# Verification of the traceback's eviction rules: the BG_SEQCHECK + BG_FIN_DEBUG build
# (exp/seqdbg.so) prints a BGDBG line whenever a helper re-assigned a slot during the walker's
# decode.  The metric bench, C3 and the traceback-heavy GPU tests; counts the lines.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/seq; export TMPDIR=/tmp
cp biogarden_amd/libbiogarden_gpu.so /tmp/lib_tree.so
cp exp/seqdbg.so biogarden_amd/libbiogarden_gpu.so
O=gpurun_out/seq
timeout -k 10 200 python bench.py --no-cpu --no-h2h --configs C3 > $O/bench.out 2> $O/bench.err; r1=$?
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py -q -s -m gpu --timeout 200 --timeout-method thread > $O/tests.out 2>&1; r2=$?
cp /tmp/lib_tree.so biogarden_amd/libbiogarden_gpu.so
echo "bench rc=$r1 tests rc=$r2 $(tail -1 $O/tests.out)"
echo "re-assigned slots during a decode: $(cat $O/bench.out $O/tests.out | grep -c 'BGDBG.*re-assigned')"
echo "other BGDBG lines: $(cat $O/bench.out $O/tests.out | grep BGDBG | grep -vc 're-assigned')"
