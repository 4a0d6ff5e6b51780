# Round 6: strip height for M's strong-scaling shares (32 / 64 pairs per GPU) after the border code.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r06/${1:-share_rs}; mkdir -p $O; export TMPDIR=/tmp
for p in ${PS:-32 64}; do
  for R in ${RS:-0 3 4 5 8}; do
    timeout -k 10 240 python bench.py --pairs $p --R $R --steps 20 --warmup 3 --no-cpu --configs '' --no-affine --no-h2h --no-steady > $O/p${p}_R$R.json 2> $O/p${p}_R$R.err || { tail -5 $O/p${p}_R$R.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/p${p}_R$R.json')); k=d['config']['kernel']; print($p, $R, d['value'], d['ms_per_step'], 'R', k['R'], 'W', k['waves'], 'wide', k['wide'], 'split', k['split'], 'dp', d['roofline']['dp_ms'], 'fin', d['roofline']['finish_ms'])"
  done
done
