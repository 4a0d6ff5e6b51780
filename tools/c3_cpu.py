#!/usr/bin/env python3
"""C3 at full size against the CPU oracle, on the GPU box (the reference's six full
matrices need ~150 GB of host RAM for 100 kbp x 100 kbp, so this runs only where MemAvailable
>= 160 GB).

One process: the GPU aligns C3 (tools/workloads.c3_pair, semiglobal blosum62 -1/-2) through the
product path; then the oracle (oracle/refcpu.c, reference-faithful: a fresh SequenceAligner
resizes to exactly (n1+1) x (n2+1), aligner.rs:92-94) aligns the same pair on ONE core, timed —
the measured CPU baseline of C3 — and its score and both aligned strings are compared with the
GPU's byte for byte.  Writes one JSON line.

    python tools/c3_cpu.py [--out FILE]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def mem_available_gib():
    with open("/proc/meminfo") as f:
        for line in f:
            if line.startswith("MemAvailable"):
                return int(line.split()[1]) / 2 ** 20
    return 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from tools import workloads
    (s1, s2), = workloads.c3_pair()
    avail = mem_available_gib()
    rec = {"config": "C3", "workload": workloads.DESCRIPTION["C3"], "cells": len(s1) * len(s2),
           "mem_available_gib": round(avail, 1)}
    from biogarden_amd.alignment import score
    from biogarden_amd.alignment.aligner import SequenceAligner
    al = SequenceAligner(0)
    t0 = time.perf_counter()
    r, = al.align_batch("semiglobal", [(s1, s2)], score.blosum62, -1, -2)
    rec["gpu_one_call_s"] = round(time.perf_counter() - t0, 3)
    al.close()
    if avail < 160:
        rec["cpu"] = "skipped: MemAvailable %.0f GiB < 160 GiB (the reference's 15 B/cell)" % avail
    else:
        from oracle import refcpu
        t0 = time.perf_counter()
        st, sc, o1, o2 = refcpu.Aligner(exact=False).align("semiglobal", s1, s2, "blosum62", -1, -2)
        secs = time.perf_counter() - t0
        rec.update({"cpu_seconds": round(secs, 2), "cpu_gcups_one_core": round(rec["cells"] / secs / 1e9, 4),
                    "cpu_kind": "port (oracle/refcpu.c, reference-faithful six full matrices, 1 core, "
                                "allocation and fill included)",
                    "status": [st, r.status], "score": [sc, r[0]],
                    "strings_equal": (o1, o2) == (bytes(r[1].chain), bytes(r[2].chain)),
                    "aligned_len": len(o1)})
    line = json.dumps(rec)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
