cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python tools/configs.py C2 C5 C4 --pipeline 3 --check 8 2>&1 | tail -3 || exit 1
BG_FIN_WAVES=4 BG_FIN_SLOTS=0 timeout -k 10 200 python tools/configs.py C4 --pipeline 3 2>&1 | tail -1
