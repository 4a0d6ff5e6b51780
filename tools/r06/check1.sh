# Round 6, first check: the new and changed GPU tests (async compact export, grouped batches with
# empty pairs, options instead of environment knobs, bounded traceback waits), the strong-scaling
# shares of M on one GPU, and a two-rank gloo rehearsal of bench.py --gpus 2 (ranks share the GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-r06/check1}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_export.py tests/test_gpu_grouped.py tests/test_gpu_split.py "tests/test_gpu_configs.py::test_traceback_walker_self_service" tests/test_gpu_parity.py::test_traceback_async_matches_barriers_and_oracle > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for p in 32 64 128 256; do
  timeout -k 10 240 python bench.py --pairs $p --steps 20 --warmup 3 --no-cpu --configs '' --no-affine --no-h2h --no-steady > $O/p$p.json 2> $O/p$p.err || { tail -20 $O/p$p.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/p$p.json')); print($p, d['value'], d['ms_per_step'], d['config']['kernel'], d['roofline']['dp_ms'], d['roofline']['finish_ms'])"
done
BG_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 6 --warmup 2 --no-h2h --no-affine --configs '' > $O/n2.json 2> $O/n2.err || { tail -20 $O/n2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/n2.json')); print({k: d.get(k) for k in ('value','n_gpus','ranks','scaling','ms_per_step','weak','gathered_expand','all_status_ok','devices','collectives')})"
