#!/bin/bash
# Round 5: the C ABI's multi-device group on the one-GPU box — its tests, then bench --group with
# one member and with two virtual members on device 0 (RCCL self-send), M's pairs per member.
set -o pipefail
out=gpurun_out/r05/${1:-group}
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_group.py tests/test_gpu_export.py tests/test_gpu_stream.py > $out/tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --group --gpus 1 --steps 10 --warmup 2 > $out/group1.json 2> $out/group1.err || exit 2
timeout -k 10 300 python3 bench.py --group --group-devices 0,0 --steps 10 --warmup 2 > $out/group00.json 2> $out/group00.err || exit 3
