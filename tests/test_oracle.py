"""The CPU oracle (oracle/refcpu.c) against every golden the reference's own tests hold.

This pins the restatement before it is trusted as the GPU checker: the 5 integration goldens
(tests/integration.rs:234-312 + tests/data/{input,output}/*_alignment.fasta) and the 5 aligner
doctests must be reproduced byte for byte, by both the reference-faithful (fresh 1024x1024
scratch) and the exact-size aligner.
"""
import json
import os

import pytest

from conftest import GOLDEN, REF_FIX, REFERENCE_DOCTESTS, REFERENCE_GOLDENS, read_fasta


@pytest.mark.parametrize("mode,scoring,a,b,expected", REFERENCE_GOLDENS)
@pytest.mark.parametrize("exact", [False, True])
def test_integration_goldens(oracle, mode, scoring, a, b, expected, exact):
    inp = read_fasta(os.path.join(REF_FIX, "input", "%s_alignment.fasta" % mode))
    out = read_fasta(os.path.join(REF_FIX, "output", "%s_alignment.fasta" % mode))
    st, score, a1, a2 = oracle.align(mode, inp[0][1], inp[1][1], scoring, a, b, exact=exact)
    assert st == 0
    assert score == expected
    assert a1 == out[0][1]
    assert a2 == out[1][1]


@pytest.mark.parametrize("case", REFERENCE_DOCTESTS, ids=lambda c: c[0])
def test_doctests(oracle, case):
    mode, s1, s2, scoring, a, b, exp, e1, e2 = case
    for exact in (False, True):
        st, score, a1, a2 = oracle.align(mode, s1, s2, scoring, a, b, exact=exact)
        assert (st, score, a1, a2) == (0, exp, e1, e2)


def test_semiglobal_prefix_drop(oracle):
    # the row case stopping at l == 0 drops seq1's prefix "GG"
    assert oracle.align("semiglobal", b"GGACGT", b"ACGTCC", "unit", -1, -1) == \
        (0, 4, b"ACGT--", b"ACGTCC")


def test_reference_errors(oracle):
    assert oracle.align("global", b"AC", b"AC", "unit", 1, -1)[0] == 1      # InvalidArgumentRange
    assert oracle.align("local", b"AC", b"AC", "unit", -1, 2)[0] == 1
    assert oracle.align("fitting", b"A", b"AC", "unit", -1, -1)[0] == 2     # InvalidInputSize
    assert oracle.align("semiglobal", b"AC", b"AC", "unit", 1, 1)[0] == 0   # no validation
    assert oracle.align("global", b"Ac", b"AC", "unit", -1, -1)[0] == 3     # score panic
    # len == buffer dim on a fresh (1024x1024) aligner panics; the exact aligner answers
    s = b"A" * 1024
    assert oracle.align("global", s, b"AC", "unit", -1, -1)[0] == 4
    assert oracle.align("global", s, b"AC", "unit", -1, -1, exact=True)[0] == 0


def test_tables_agree():
    """Product tables (bg_tables.inc), oracle tables and the golden JSON are one data set."""
    from oracle import refcpu
    with open(os.path.join(GOLDEN, "score_tables.json")) as f:
        gold = json.load(f)["tables"]
    for name in ("blosum62", "pam250", "unit"):
        sc = refcpu.scoring(name)
        for r in range(26):
            for c in range(26):
                assert sc.table[r * 32 + c] == gold[name][r][c]
    # product decode (pure host code, no GPU needed)
    from biogarden_amd import _native
    for name, which in (("blosum62", 0), ("pam250", 1), ("unit", 2)):
        sc = _native.builtin_scoring(which)
        assert sc.alphabet_size == 26
        for r in range(26):
            for c in range(26):
                assert sc.table[r * 32 + c] == gold[name][r][c], (name, r, c)
        assert sc.code[ord("A")] == 0 and sc.code[ord("Z")] == 25 and sc.code[ord("a")] == 0xFF


def test_blosum62_dna_block():
    """the DNA sub-block of the reference BLOSUM62."""
    with open(os.path.join(GOLDEN, "score_tables.json")) as f:
        b = json.load(f)["tables"]["blosum62"]
    ix = {ch: ord(ch) - 65 for ch in "ACGT"}
    want = {"AA": 4, "CC": 9, "GG": 6, "TT": 5, "AC": 0, "AG": 0, "AT": 0, "CG": -3, "CT": -1,
            "GT": -2}
    for k, v in want.items():
        assert b[ix[k[0]]][ix[k[1]]] == v == b[ix[k[1]]][ix[k[0]]]


# ------------------------------------------------------------------ edit distance / LCS / SCS
# tests/integration.rs:69-74 (299), :135-149 (fixtures) and the doctests seq.rs:97-104,
# patterns.rs:73-80, 190-196

def test_edit_distance_golden(oracle):
    inp = read_fasta(os.path.join(REF_FIX, "input", "edit_distance.fasta"))
    assert oracle.edit_distance(inp[0][1], inp[1][1]) == 299
    assert oracle.edit_distance(b"ACTGGATTC", b"ACGT") == 5


def test_lcs_scs_goldens(oracle):
    inp = read_fasta(os.path.join(REF_FIX, "input", "longest_common_subseq.fasta"))
    out = read_fasta(os.path.join(REF_FIX, "output", "longest_common_subseq.fasta"))
    assert oracle.longest_common_subsequence(inp[0][1], inp[1][1]) == out[0][1]
    inp = read_fasta(os.path.join(REF_FIX, "input", "shortest_common_superseq.fasta"))
    out = read_fasta(os.path.join(REF_FIX, "output", "shortest_common_superseq.fasta"))
    assert oracle.shortest_common_supersequence(inp[0][1], inp[1][1]) == out[0][1]
    assert oracle.longest_common_subsequence(b"AACCTTGG", b"ACACTGTGA") == b"ACCTGG"
    assert oracle.shortest_common_supersequence(b"TGCATA", b"ATCTGAT") == b"ATGCATGAT"


def test_edit_distance_small_cases(oracle):
    assert oracle.edit_distance(b"", b"") == 0
    assert oracle.edit_distance(b"", b"ACG") == 3
    assert oracle.edit_distance(b"ACGT", b"") == 4
    assert oracle.edit_distance(b"kitten", b"sitting") == 3


def test_scs_merge_matches_oracle(oracle):
    """The product's host-side supersequence merge (patterns.rs:198-235) around the oracle's LCS."""
    import random

    from biogarden_amd.processing.patterns import _merge
    rng = random.Random(5)
    for _ in range(200):
        a = bytes(rng.choice(b"ACGT") for _ in range(rng.randint(0, 40)))
        b = bytes(rng.choice(b"ACGT") for _ in range(rng.randint(0, 40)))
        lcs = oracle.longest_common_subsequence(a, b)
        assert _merge(a, b, lcs) == oracle.shortest_common_supersequence(a, b)


def test_C1_derived_golden_reproduced(oracle):
    """The committed C1 golden (oracle-derived, tools/make_derived_goldens.py) is what the
    reference-faithful oracle computes for examples/from_file.rs's call."""
    with open(os.path.join(GOLDEN, "derived", "C1_semiglobal_blosum62_o1_e2.json")) as f:
        gold = json.load(f)
    assert gold["derived"] is True
    inp = read_fasta(os.path.join(REF_FIX, "input", "semiglobal_alignment.fasta"))
    assert (len(inp[0][1]), len(inp[1][1])) == (gold["len1"], gold["len2"]) == (9559, 8457)
    st, score, a1, a2 = oracle.align("semiglobal", inp[0][1], inp[1][1], "blosum62", -1, -2)
    assert (st, score, a1, a2) == (0, gold["score"], gold["aligned1"].encode(), gold["aligned2"].encode())


def test_reused_aligner_scratch_model(oracle):
    """resize_buffers only on a strict overflow, both dims reset (aligner.rs:92-94, 594-602):
    a length equal to the current dim panics, one beyond it resizes; errors return first."""
    al = oracle.Aligner()
    assert al.buffer_size() == (1024, 1024)
    assert al.align("global", b"A" * 2000, b"C" * 10, "unit", -1, -1)[0] == 0
    assert al.buffer_size() == (2001, 11)
    assert al.align("global", b"A" * 1024, b"C" * 11, "unit", -1, -1)[0] == 4   # col 11 == dim
    assert al.buffer_size() == (2001, 11)
    assert al.align("global", b"A" * 1024, b"C" * 12, "unit", -1, -1)[0] == 0   # 12 > 11: resize
    assert al.buffer_size() == (1025, 13)
    assert al.align("global", b"A" * 5000, b"C", "unit", 1, -1)[0] == 1         # error, no resize
    assert al.buffer_size() == (1025, 13)
    d = oracle.Aligner(dims=(1025, 13))
    assert d.buffer_size() == (1025, 13)
    assert d.align("global", b"A" * 1025, b"C", "unit", -1, -1)[0] == 4
