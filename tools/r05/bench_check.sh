#!/bin/bash
# Round 5: the default bench as the driver runs it (N = 1), then through torch.distributed.run
# with one rank (the N > 1 code path, RCCL world of 1).
set -o pipefail
out=gpurun_out/r05/${1:-bcheck}
mkdir -p $out
timeout -k 10 600 python bench.py > $out/default.json 2> $out/default.err || { tail -20 $out/default.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-h2h --configs "" > $out/dist1.json 2> $out/dist1.err || { tail -20 $out/dist1.err; exit 2; }
