# rocprofv3 kernel-trace summary of the SURVEY §8(d) configs (default C2 C5), no PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_cfg
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg -o run --output-format csv -- python3 tools/configs.py ${CFGS:-C2 C5} --steps 5 --pipeline 3 > gpurun_out/prof_cfg/configs.log 2>&1
rc=$?
find gpurun_out/prof_cfg -name "*stats*.csv"
cat gpurun_out/prof_cfg/configs.log | grep config
exit $rc
