#!/usr/bin/env python3
"""Per-wave strip timeline of the DP kernel for the first pair of a batch (BG_DEBUG=dp).

    BG_DEBUG=dp python tools/dp_timeline.py [--pairs 256] [--len 10000] [--R 8 --waves 16]

One execute at pipeline depth 1 after a warm-up; the host prints, for each wave of pair 0, the
strip it ran last in round 0, its start / first-chunk / end times and the cycles it spent waiting.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from biogarden_amd import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=256)
    ap.add_argument("--len", type=int, default=10000)
    ap.add_argument("--R", type=int, default=0)
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--mode", default="semiglobal")
    ap.add_argument("--a", type=int, default=-1)
    ap.add_argument("--b", type=int, default=-2)
    args = ap.parse_args()
    rng = np.random.default_rng(7)
    dna = np.frombuffer(b"ACGT", dtype=np.uint8)
    pairs = [(dna[rng.integers(0, 4, args.len)].tobytes(), dna[rng.integers(0, 4, args.len)].tobytes())
             for _ in range(args.pairs)]
    h = _native.Handle(0)
    if args.R:
        h.set_tuning(R=args.R, waves=args.waves)
    h.set_pipeline(1)
    sc = _native.builtin_scoring(_native.BG_BLOSUM62)
    for it in range(2):
        h.prepare(args.mode, pairs, sc, args.a, args.b)
        t = time.perf_counter()
        h.execute()
        h.synchronize()
        dt = time.perf_counter() - t
        print(f"run {it}: {dt * 1e3:.2f} ms, stats {h.stats()}", file=sys.stderr)
        h.fetch()
    h.close()


if __name__ == "__main__":
    main()
