# PMC passes (tools/pmc.sh) for the bench's metric leg (M, -1/-2) and its affine leg (MA, -11/-1),
# each summarised into profiles/pmc_<workload>.json by tools/pmc_traffic.py.
cd $GRAFT_REPO_ROOT
mkdir -p profiles
export PASSES="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAVE_CYCLES,GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE"
BENCH_ARGS="--no-affine --no-h2h --R 8 --waves 16" bash tools/pmc.sh > /dev/null || exit 1
python3 tools/pmc_traffic.py gpurun_out/pmc/summary.json semiglobal_256x10000x10000_blosum62_o1_e2 6405120000 8 16 | head -12 || exit 1
mv gpurun_out/pmc gpurun_out/pmc_M
BENCH_ARGS="--no-affine --no-h2h --open -11 --extend -1 --R 4 --waves 16" bash tools/pmc.sh > /dev/null || exit 1
python3 tools/pmc_traffic.py gpurun_out/pmc/summary.json semiglobal_256x10000x10000_blosum62_o11_e1 12805120000 4 16 | head -12 || exit 1
mv gpurun_out/pmc gpurun_out/pmc_MA
mkdir -p gpurun_out/pmcout && cp profiles/pmc_*.json gpurun_out/pmcout/
