# Strong-scaling shares of M on one GPU: --pairs P of 10k x 10k (P = 256/G for G = 8,4,2,1):
# the per-GPU step of the strong form without the gather.  usage: bash tools/r06/strong_shares.sh <out>
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-shares}; mkdir -p $O; export TMPDIR=/tmp
for p in 32 64 128 256; do
  timeout -k 10 240 python bench.py --pairs $p --steps 20 --warmup 3 --no-cpu --configs '' --no-affine --no-h2h --no-steady > $O/p$p.json 2> $O/p$p.err || { tail -20 $O/p$p.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/p$p.json')); print($p, d['value'], d['ms_per_step'], d['config']['kernel'], d['roofline']['dp_ms'], d['roofline']['finish_ms'])"
done
