set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
BG_FINISH_TIMING=1 timeout -k 10 200 python tools/configs.py C3 --steps 3 --timing > gpurun_out/c3_fin_timing.txt 2>&1 || exit 4
grep -i "finish timing" gpurun_out/c3_fin_timing.txt | tail -2; tail -1 gpurun_out/c3_fin_timing.txt
