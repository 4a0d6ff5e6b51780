#!/usr/bin/env python3
"""Writes tests/golden/derived/C1_semiglobal_blosum62_o1_e2.json: the oracle's output for
BASELINE config 1 — semiglobal_alignment on the reference's tests/data/input/
semiglobal_alignment.fasta (records 0 and 1, 9559 x 8457) with score::blosum62, a = -1, b = -2,
the parameters of the reference's examples/from_file.rs:14-31.

DERIVED, not reference-produced: the reference publishes no output for these parameters (its
golden for this file uses unit -1/-1, tests/integration.rs:298-312).  The oracle that produced
it (oracle/refcpu.c, reference-faithful aligner) is pinned by the reference's own goldens and
doctests (tests/test_oracle.py); SURVEY.md §8(c) asks for exactly this derived golden.

    python tools/make_derived_goldens.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import REF_FIX, read_fasta  # noqa: E402
from oracle import refcpu  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "derived", "C1_semiglobal_blosum62_o1_e2.json")


def main():
    recs = read_fasta(os.path.join(REF_FIX, "input", "semiglobal_alignment.fasta"))
    s1, s2 = recs[0][1], recs[1][1]
    al = refcpu.Aligner(exact=False)            # SequenceAligner::new(), as from_file.rs does
    st, score, o1, o2 = al.align("semiglobal", s1, s2, "blosum62", -1, -2)
    assert st == 0, st
    doc = {
        "derived": True,
        "note": "oracle output (oracle/refcpu.c, reference-faithful), NOT produced by the "
                "reference itself; see tools/make_derived_goldens.py",
        "config": "C1: semiglobal_alignment, blosum62, a=-1, b=-2 (examples/from_file.rs:14-31)",
        "input": "tests/golden/reference_fixtures/input/semiglobal_alignment.fasta records 0,1",
        "len1": len(s1), "len2": len(s2),
        "score": score, "aligned1": o1.decode(), "aligned2": o2.decode(),
    }
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print("wrote", OUT, "score", score, "len", len(o1))


if __name__ == "__main__":
    main()
