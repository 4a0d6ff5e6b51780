# metric bench + finish-kernel timing (cycles per pair) of the metric and C2/C5
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
echo "== bench"; timeout -k 10 200 python bench.py --no-cpu --no-h2h 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['config']['kernel'], d['roofline']['kernel_ms'], d['roofline']['finish_ms'])" || exit 1
echo "== finish timing (metric, alone)"; timeout -k 10 200 python tools/finish_timing.py 2>&1 | tail -2 || exit 1
timeout -k 10 200 python tools/configs.py C2 C5 --R 4 --pipeline 1 --timing 2>&1 | tail -4
timeout -k 10 200 python tools/configs.py C2 C5 C4 --pipeline 3 2>&1 | tail -3
