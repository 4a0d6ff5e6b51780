# Round 6: SPAN geometry sweep at M's strong-scaling shares (128 / 64 pairs: 2 / 4 GPUs), R x W
# forced (BG_OPTIONS span=1, bench --R --waves), plus 32 pairs as SPAN with the split traceback.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-r06/span_sweep}; mkdir -p $O; export TMPDIR=/tmp
one() {  # pairs R W options tag
  BG_OPTIONS="$4" timeout -k 10 120 python bench.py --pairs $1 --R $2 --waves $3 --steps 20 --warmup 3 --no-cpu --configs '' --no-affine --no-h2h --no-steady > $O/$5.json 2> $O/$5.err || { tail -5 $O/$5.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$5.json')); k=d['config']['kernel']; print('$5', d['value'], d['ms_per_step'], 'R', k['R'], 'W', k['waves'], 'wide', k['wide'], 'split', k['split'], 'dp', d['roofline']['dp_ms'], 'fin', d['roofline']['finish_ms'])"
}
for p in 128 64; do
  for R in 3 4 5 8 10; do
    for W in 4 8 12 16; do
      one $p $R $W "span=1" p${p}_R${R}_W${W} || exit 1
    done
  done
done
for R in 3 5 8; do for W in 4 8; do one 32 $R $W "span=1,split=1" p32_R${R}_W${W}_split || exit 1; one 32 $R $W "span=1" p32_R${R}_W${W} || exit 1; done; done
