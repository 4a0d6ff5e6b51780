set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-r06/dbg}; mkdir -p $O
for m in "global -2,-2" "semiglobal -1,-2" "overlap -2,-2" "fitting -1,-2"; do
  timeout -k 10 120 python3 tools/r06/dbg_global.py $m >> $O/dbg.txt 2>&1 || { tail -20 $O/dbg.txt; exit 1; }
done
cat $O/dbg.txt
