# Round 6: the N > 1 strong-form bench rehearsed on the one-GPU box (two gloo ranks sharing the
# GPU), M and C4, after the one-wave export scan.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r06/${1:-n2}; mkdir -p $O; export TMPDIR=/tmp
BG_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 6 --warmup 2 --no-h2h > $O/n2.json 2> $O/n2.err || { tail -20 $O/n2.err; exit 1; }
python3 tools/summ_bench.py $O/n2.json
python3 -c "import json; d=json.loads(open('$O/n2.json').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('n_gpus','ranks','rehearsal','collectives','value','ms_per_step','strong','weak','all_status_ok')})"
BG_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 3 --warmup 1 --config C4 > $O/n2_c4.json 2> $O/n2_c4.err || { tail -20 $O/n2_c4.err; exit 2; }
python3 -c "import json; d=json.loads(open('$O/n2_c4.json').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('n_gpus','ranks','value','ms_per_step','all_status_ok')})"
