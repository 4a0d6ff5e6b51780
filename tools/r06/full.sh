# Round 6: the whole GPU suite, the default bench (configs, affine, host-to-host, CPU baseline
# included), smoke(), and the strong-scaling shares of M (32 / 64 / 128 pairs: one GPU's share at
# 8 / 4 / 2 GPUs).  Stops at the first failure.  usage: bash tools/r06/full.sh <out>
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-r06/full}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 2; }
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
python3 tools/summ_bench.py $O/bench.json
for p in 128 64 32; do
  timeout -k 10 240 python bench.py --pairs $p --steps 20 --warmup 3 --no-cpu --configs '' --no-affine --no-h2h --no-steady > $O/p$p.json 2> $O/p$p.err || { tail -20 $O/p$p.err; exit 4; }
  python3 -c "import json; d=json.load(open('$O/p$p.json')); k=d['config']['kernel']; print($p, d['value'], d['ms_per_step'], 'R', k['R'], 'W', k['waves'], 'wide', k['wide'], 'split', k['split'], 'dp', d['roofline']['dp_ms'], 'fin', d['roofline']['finish_ms'])"
done
