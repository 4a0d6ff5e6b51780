#!/usr/bin/env python3
"""Finish-workgroup geometry vs pairs per CU: GCUPS of C2-shaped (local 1k x 1k DNA, -11/-1) and
C5-shaped (global protein, -11/-1) batches at several batch sizes, for the current fin_geom
(or BG_FIN_WAVES / BG_FIN_SLOTS from the environment).  python tools/fin_geom_np.py"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from biogarden_amd import _native  # noqa: E402

DNA = np.frombuffer(b"ACGT", dtype=np.uint8)
PROT = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", dtype=np.uint8)


def run(h, mode, pairs, a, b, steps=12):
    sc = _native.builtin_scoring(_native.BG_BLOSUM62)
    h.prepare(mode, pairs, sc, a, b)
    h.execute(); h.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        h.execute()
    h.synchronize()
    el = (time.perf_counter() - t) / steps
    h.fetch()
    return sum(len(x) * len(y) for x, y in pairs) / el / 1e9


def main():
    rng = np.random.default_rng(3)
    h = _native.Handle(0)
    tag = "waves=%s slots=%s" % (os.environ.get("BG_FIN_WAVES", "-"), os.environ.get("BG_FIN_SLOTS", "-"))
    for n in (1024, 4096):
        pairs = [(DNA[rng.integers(0, 4, 1000)].tobytes(), DNA[rng.integers(0, 4, 1000)].tobytes()) for _ in range(n)]
        print(json.dumps({"geom": tag, "shape": "C2", "pairs": n, "gcups": round(run(h, "local", pairs, -11, -1), 1)}), flush=True)
    for n in (1024, 4080):
        pairs = []
        for _ in range(n):
            n1, n2 = (int(x) for x in rng.integers(64, 4001, 2))
            pairs.append((PROT[rng.integers(0, 20, n1)].tobytes(), PROT[rng.integers(0, 20, n2)].tobytes()))
        print(json.dumps({"geom": tag, "shape": "C5", "pairs": n, "gcups": round(run(h, "global", pairs, -11, -1), 1)}), flush=True)
    h.close()


if __name__ == "__main__":
    main()
