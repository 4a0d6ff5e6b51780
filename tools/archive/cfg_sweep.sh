cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python tools/configs.py C2 C5 --R 4 --pipeline 1 --timing > gpurun_out/cfgT.log 2>&1
timeout -k 10 200 python tools/configs.py C2 C5 --pipeline 3 >> gpurun_out/cfgT.log 2>&1
cat gpurun_out/cfgT.log
