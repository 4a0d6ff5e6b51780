# Round 6: SPAN parity (fewer pairs than CUs, pairs over groups of many-wave workgroups), the
# traceback tests touched by the bounded waits, then M at 256 pairs and the strong-scaling shares
# (32 / 64 / 128 pairs) with the automatic plan and with span = 0 (BG_OPTIONS) for A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-r06/check2}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_span.py "tests/test_gpu_configs.py::test_traceback_walker_self_service" tests/test_gpu_export.py::test_compact_export_async_pipelined > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for p in 256 128 64 32; do
  for opt in "" "span=0"; do
    BG_OPTIONS="$opt" timeout -k 10 240 python bench.py --pairs $p --steps 20 --warmup 3 --no-cpu --configs '' --no-affine --no-h2h --no-steady > $O/p${p}_${opt:-auto}.json 2> $O/p${p}_${opt:-auto}.err || { tail -20 $O/p${p}_${opt:-auto}.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/p${p}_${opt:-auto}.json')); k=d['config']['kernel']; print($p, '${opt:-auto}', d['value'], d['ms_per_step'], 'R', k['R'], 'W', k['waves'], 'wide', k['wide'], 'dp', d['roofline']['dp_ms'], 'fin', d['roofline']['finish_ms'])"
    [ "$p" = 256 ] && break
  done
done
