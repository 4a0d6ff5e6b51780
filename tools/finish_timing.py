#!/usr/bin/env python3
"""Per-pair cycle breakdown of the finish kernel (BG_DEBUG=finish): walk total, jumper blocks,
misses (window loads / chunk recomputation), chunks recomputed.
    python tools/finish_timing.py [pairs] [ckpt 0/1] [R W]"""
import os
import sys

os.environ["BG_DEBUG"] = "finish"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from biogarden_amd import _native  # noqa: E402

npairs = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ck = int(sys.argv[2]) if len(sys.argv) > 2 else 1
h = _native.Handle(0)
h.set_pipeline(1)
h.set_kernel_options(True, bool(ck))
if len(sys.argv) > 4:
    h.set_tuning(int(sys.argv[3]), int(sys.argv[4]))
L = int(os.environ.get("LEN", "10000"))
pairs = bench.make_pairs(npairs, L, L, bench.SEED)
ga, gb = (int(x) for x in os.environ.get("GAPS", "-1,-2").split(","))
h.prepare("semiglobal", pairs, _native.builtin_scoring(_native.BG_BLOSUM62), ga, gb)
h.execute()
h.fetch()
h.profile_begin()
h.execute()
dp, fin, n = h.profile_end()
h.fetch()
st = h.stats()
print("R", st["R"], "W", st["waves"], "ckpt", st["checkpoint"], "dp_ms %.3f finish_ms %.3f" % (dp, fin), flush=True)
