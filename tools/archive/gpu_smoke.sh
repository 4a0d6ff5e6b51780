set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "golden or doctest or errors" > gpurun_out/t1.log 2>&1
echo "exit $?" >> gpurun_out/t1.log
tail -30 gpurun_out/t1.log
