#!/usr/bin/env python3
"""Per-GPU throughput of the SURVEY.md §8(d) configurations (the metric M is bench.py's).

    python tools/configs.py [C2 C3 C4 C5 ...] [--steps K] [--check N]

C4 and C5 run the share of one GPU out of 8 (the batch is sharded over ranks, weak per rank).
Inputs are synthetic as §8(d) describes (uniform DNA / protein, 2 % substituted reads).
--check N compares the first N pairs' scores against the CPU oracle (slow for big pairs).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DNA = np.frombuffer(b"ACGT", dtype=np.uint8)
PROT = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", dtype=np.uint8)


def rand_seq(rng, alpha, n):
    return alpha[rng.integers(0, len(alpha), n)].tobytes()


def config(name, rng):
    if name == "C2":      # 1024 x (1000 x 1000) local DNA, blosum62, -11/-1
        pairs = [(rand_seq(rng, DNA, 1000), rand_seq(rng, DNA, 1000)) for _ in range(1024)]
        return "local", pairs, -11, -1
    if name == "C3":      # 1 x (100 000 x 100 000) semiglobal, blosum62, -1/-2
        return "semiglobal", [(rand_seq(rng, DNA, 100000), rand_seq(rng, DNA, 100000))], -1, -2
    if name == "C4":      # 65 536 reads (150 bp, 2 % substitutions) vs 64 refs of 10 kbp; 1/8
        refs = [rand_seq(rng, DNA, 10000) for _ in range(8)]
        pairs = []
        for r in refs:
            ra = np.frombuffer(r, dtype=np.uint8)
            for _ in range(1024):
                o = int(rng.integers(0, 10000 - 150))
                read = ra[o:o + 150].copy()
                m = rng.random(150) < 0.02
                read[m] = DNA[rng.integers(0, 4, int(m.sum()))]
                pairs.append((read.tobytes(), r))
        return "semiglobal", pairs, -1, -2
    if name == "C5":      # all-vs-all 256 proteins U[64, 4000], global, blosum62, -11/-1; 1/8
        prots = [rand_seq(rng, PROT, int(rng.integers(64, 4001))) for _ in range(256)]
        allp = [(prots[i], prots[j]) for i in range(256) for j in range(i + 1, 256)]
        return "global", allp[0::8], -11, -1
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["C2", "C4", "C5", "C3"])
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--check", type=int, default=0)
    ap.add_argument("--pipeline", type=int, default=3)
    ap.add_argument("--R", type=int, default=0)
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--kernel-options", type=int, default=7)
    ap.add_argument("--timing", action="store_true", help="finish-kernel cycle breakdown (stderr)")
    args = ap.parse_args()
    if args.timing:
        os.environ["BG_FINISH_TIMING"] = "1"
    from biogarden_amd import _native
    h = _native.Handle(0)
    h.set_pipeline(args.pipeline)
    h.set_tuning(args.R, args.waves)
    h.set_kernel_options(bool(args.kernel_options & 1), bool(args.kernel_options & 2),
                         bool(args.kernel_options & 4))
    sc = _native.builtin_scoring(_native.BG_BLOSUM62)
    for i, name in enumerate(args.configs):
        rng = np.random.default_rng(0xB10A11F0 + int(name[1:]))
        mode, pairs, a, b = config(name, rng)
        t0 = time.perf_counter()
        h.prepare(mode, pairs, sc, a, b)
        prep = time.perf_counter() - t0
        st = h.stats()
        h.execute()
        h.synchronize()
        h.profile_begin()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            h.execute()
        h.synchronize()
        el = (time.perf_counter() - t0) / args.steps
        dp, fin, n = h.profile_end()
        res = h.fetch()
        bad = sum(1 for r in res if r["status"] not in (0, 4))
        line = {"config": name, "mode": mode, "pairs": len(pairs), "cells": st["cells"],
                "gcups": round(st["cells"] / el / 1e9, 2), "ms_per_step": round(el * 1e3, 3),
                "dp_ms": round(dp, 3), "finish_ms": round(fin, 3), "prepare_s": round(prep, 3),
                "R": st["R"], "waves": st["waves"], "affine": st["affine"], "tagged": st["tagged"],
                "dna": st["dna"], "bad_status": bad}
        if args.check:
            from oracle import refcpu
            k = min(args.check, len(pairs))
            secs, scores, sts = refcpu.align_batch(mode, pairs[:k], "blosum62", a, b,
                                                   nthreads=min(16, os.cpu_count() or 1), exact=True)
            line["oracle_match"] = "%d/%d" % (sum(int(s == r["score"]) for s, r in zip(scores, res)), k)
            line["oracle_gcups"] = round(sum(len(x) * len(y) for x, y in pairs[:k]) / secs / 1e9, 4)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
