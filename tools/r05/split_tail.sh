#!/bin/bash
# Round 5: the post-DP exit pass skips the start strip's items after the capture item (ADVICE
# r04): the split tests, the full-size C3 string test, and C3's single-alignment wall.
set -o pipefail
out=gpurun_out/r05/${1:-splittail}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_zz_gpu_c3_full.py -m gpu -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|FAIL" $out/tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/configs.py C3 --steps 12 --single 5 > $out/c3.txt 2>&1 || exit 2
