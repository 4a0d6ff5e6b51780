# Geometry re-check after a kernel change: MA and M through bench.py, C2 / C5 through configs.py
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
echo "== MA"; OPEN=-11 EXT=-1 STEPS=8 RWS="0,0 4,8 4,16 8,8 8,16 2,16" bash tools/aff_sweep.sh || exit 1
echo "== M"; OPEN=-1 EXT=-2 STEPS=10 RWS="0,0 5,16 10,16 4,16 8,12" bash tools/aff_sweep.sh || exit 1
for cfg in C5 C2; do
  for rw in 0,0 2,2 2,4 2,8 4,2 4,4; do
    IFS=, read -r RR WW <<< "$rw"
    echo -n "$cfg $rw "
    timeout -k 10 120 python tools/configs.py $cfg --R $RR --waves $WW --steps 12 2>/dev/null | cut -c1-170 || exit 1
  done
done
