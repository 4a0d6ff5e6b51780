#!/usr/bin/env python3
"""Per-GPU throughput of the SURVEY.md §8(d) configurations (the metric M is bench.py's).

    python tools/configs.py [C2 C3 C4 C5 ...] [--steps K] [--check N]

C4 and C5 are one batch over 8 GPUs: the whole job is generated
(tools/workloads.py) and LPT-sharded by cells over --world ranks (biogarden_amd.shard.lpt_shards,
the multi-GPU path's partition); this process runs --rank's shard.  Inputs are synthetic as
§8(d) describes (uniform DNA / protein, 2 % substituted reads).
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


def config(name, rng, rank=0, world=8):
    if name == "C2":      # 1024 x (1000 x 1000) local DNA, blosum62, -11/-1
        pairs = [(rand_seq(rng, DNA, 1000), rand_seq(rng, DNA, 1000)) for _ in range(1024)]
        return "local", pairs, -11, -1
    if name == "C3":      # 1 x (100 000 x 100 000) semiglobal, blosum62, -1/-2
        return "semiglobal", [(rand_seq(rng, DNA, 100000), rand_seq(rng, DNA, 100000))], -1, -2
    if name in ("C4", "C5"):  # one batch over `world` GPUs: this rank's LPT shard of the job
        from biogarden_amd.shard import lpt_shards
        from tools import workloads
        if name == "C4":      # 65 536 reads (150 bp, 2 % substitutions) vs 64 refs of 10 kbp
            mode, allp, a, b = "semiglobal", workloads.c4_pairs(), -1, -2
        else:                 # all-vs-all 256 proteins U[64, 4000], global, blosum62, -11/-1
            mode, allp, a, b = "global", workloads.c5_pairs(), -11, -1
        shards = lpt_shards([(len(x), len(y)) for x, y in allp], world)
        return mode, [allp[p] for p in shards[rank]], a, b
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
    ap.add_argument("--rank", type=int, default=0, help="C4 / C5: the shard this GPU runs")
    ap.add_argument("--world", type=int, default=8, help="C4 / C5: GPUs the job is sharded over")
    ap.add_argument("--torch-init", action="store_true", help="initialise torch on the GPU first")
    ap.add_argument("--warm-ms", type=float, default=0.0,
                    help="untimed executes for at least this long before the timed ones")
    ap.add_argument("--single", type=int, default=0,
                    help="also time N lone executes (execute + synchronize each): one alignment's wall")
    args = ap.parse_args()
    if args.timing:
        os.environ["BG_DEBUG"] = "finish"
    if args.torch_init:                  # torch's HIP runtime state first, as in bench.py
        import torch
        torch.zeros(1, device="cuda")
        torch.cuda.synchronize()
    from biogarden_amd import _native
    h = _native.Handle(0)
    h.set_pipeline(args.pipeline)
    h.set_tuning(args.R, args.waves)
    h.set_kernel_options(bool(args.kernel_options & 1), bool(args.kernel_options & 2),
                         bool(args.kernel_options & 4))
    sc = _native.builtin_scoring(_native.BG_BLOSUM62)
    for i, name in enumerate(args.configs):
        rng = np.random.default_rng(0xB10A11F0 + int(name[1:]))
        mode, pairs, a, b = config(name, rng, args.rank, args.world)
        if name in ("C4", "C5"):      # the whole job's call history (status 4, shard.call_dims)
            from biogarden_amd import shard
            from tools import workloads
            allp = workloads.job(name)[1]
            sizes = [(len(x), len(y)) for x, y in allp]
            idx = shard.lpt_shards(sizes, args.world)[args.rank]
            h.set_call_dims(shard.shard_call_dims(mode, sizes, a, b, idx))
        t0 = time.perf_counter()
        h.prepare(mode, pairs, sc, a, b)
        prep = time.perf_counter() - t0
        st = h.stats()
        h.execute()
        h.synchronize()
        tw = time.perf_counter()
        while (time.perf_counter() - tw) * 1e3 < args.warm_ms:
            h.execute()
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
        bpc = 0.25 if a >= b else 0.5          # SURVEY §8(d) algorithmic bytes per cell
        line = {"config": name, "mode": mode, "pairs": len(pairs), "cells": st["cells"],
                "algorithmic_bytes": int(st["cells"] * bpc + st["residue_bytes"]),
                "gcups": round(st["cells"] / el / 1e9, 2), "ms_per_step": round(el * 1e3, 3),
                "dp_ms": round(dp, 3), "finish_ms": round(fin, 3), "prepare_s": round(prep, 3),
                "R": st["R"], "waves": st["waves"], "affine": st["affine"], "tagged": st["tagged"],
                "dna": st["dna"], "bad_status": bad}
        if name in ("C4", "C5"):
            line["shard"] = "rank %d of %d (LPT by cells)" % (args.rank, args.world)
        if args.single:
            walls, dps, fins = [], [], []
            for _ in range(args.single):
                h.synchronize()
                t0 = time.perf_counter()
                h.execute()
                h.synchronize()
                walls.append((time.perf_counter() - t0) * 1e3)
                s2 = h.stats()
                dps.append(s2["dp_ms"])
                fins.append(s2["finish_ms"])
            walls.sort()
            line["single"] = {"wall_ms_min": round(walls[0], 3), "wall_ms_median": round(walls[len(walls) // 2], 3),
                              "dp_ms": round(sorted(dps)[len(dps) // 2], 3),
                              "finish_ms": round(sorted(fins)[len(fins) // 2], 3),
                              "gcups": round(st["cells"] / (walls[len(walls) // 2] * 1e-3) / 1e9, 2)}
            try:
                line["split_stats"] = h.split_stats()
                line["conc_diag"] = h.conc_diag()
            except Exception:                         # noqa: BLE001 (older library)
                pass
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
