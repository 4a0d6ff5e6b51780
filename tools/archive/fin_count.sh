# finish-kernel breakdown (walk cycles, misses, chunks recomputed per pair): async vs barriers
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python tools/finish_timing.py 64 2>&1 | tail -2 || exit 1
BG_FIN_SYNC=1 timeout -k 10 200 python tools/finish_timing.py 64 2>&1 | tail -2 || exit 1
