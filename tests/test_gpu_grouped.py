"""Grouped DP (bg_grp_kernel.hip, round 5): short reads that share a reference run P to a wave
(P = 4: one per 16-lane DPP row; P = 2: 32 lanes each), and the traceback recomputes a pair's
chunks as 64 / P-lane jobs (bg_finish.h recompute_grp).  Results must not change: score and both
strings against the oracle, and identical to the one-wave-per-pair path (BG_GROUPED=0) over
whole batches (bg_set_option grouped = 0), at both P and every R the planner picks ((64 / P) R >= the longest read), in the
four linear-path modes, with references shorter than a chunk, one column long, and groups with
empty rows."""
import os
import random

import pytest

from parity_util import DNA, check_batch, check_results, mutate, rand_seq, sample_indices

pytestmark = pytest.mark.gpu


def _align(mode, pairs, a, b, grouped, P=""):
    from biogarden_amd.alignment import score
    from biogarden_amd.alignment.aligner import SequenceAligner
    al = SequenceAligner(0)
    try:
        al.set_option("grouped", int(grouped) if grouped else None)
        al.set_option("group_pairs", int(P) if P else None)
        res = al.align_batch(mode, pairs, score.blosum62, a, b)
        return res, al.stats()
    finally:
        al.close()


def _key(r):
    return (r.status, r[0], bytes(r[1].chain), bytes(r[2].chain))


@pytest.mark.parametrize("P", ["4", "2"])
def test_grouped_C4_slice_matches_ungrouped(oracle, P):
    from tools import workloads as w
    pairs = w.c4_pairs(nrefs=8, reads_per_ref=131)          # 131 per reference: partial groups
    res, st = _align("semiglobal", pairs, -1, -2, "", P)
    ng = 8 * ((131 + int(P) - 1) // int(P))
    assert st["grouped"] == ng and st["group_pairs"] == int(P) and st["checkpoint"] == 1, st
    assert st["R"] == (5 if P == "2" else 10), st
    assert (st["fin_waves"], st["fin_slots"]) == (1, 6), st
    ref, st0 = _align("semiglobal", pairs, -1, -2, "0")
    assert st0["grouped"] == 0, st0
    diff = [p for p in range(len(pairs)) if _key(res[p]) != _key(ref[p])]
    assert not diff, diff[:10]
    check_results(oracle, "semiglobal", pairs, res, "blosum62", -1, -2,
                  sample=sample_indices(len(pairs), 48, 11))
    assert all(r.status == 0 and r.end[0] == 150 for r in res)


def _edge_pairs(seed, R, mode, P):
    rng = random.Random(seed)
    top = (64 // P) * R
    reflens = [1, 5, 63, 64, 65, 127, 200, 700]
    if mode == "fitting":                                   # seq2 fits in seq1 (n2 <= n1)
        reflens = [1, 2, 5, max(1, top // 4), max(1, top // 2), top - 1, top]
    pairs = []
    for n2 in reflens:
        ref = rand_seq(rng, n2, DNA)
        lo = n2 if mode == "fitting" else 1
        lens = [lo, top, top - 1, max(lo, top - 15), max(lo, top // 2), rng.randint(lo, top), rng.randint(lo, top)]
        for n1 in lens[:5 + (n2 % 3)]:                      # 5 .. 7 reads: groups with empty rows
            n1 = max(n1, lo)
            if n2 > n1 and rng.random() < 0.6:
                o = rng.randint(0, n2 - n1)
                read = (mutate(rng, ref[o:o + n1], DNA, 0.1) + rand_seq(rng, n1, DNA))[:n1]
            elif mode == "fitting" and rng.random() < 0.6:      # the reference inside the read
                o = rng.randint(0, n1 - n2)
                read = (rand_seq(rng, o, DNA) + mutate(rng, ref, DNA, 0.1) + rand_seq(rng, n1, DNA))[:n1]
            else:
                read = rand_seq(rng, n1, DNA)
            pairs.append((read, ref))
    return pairs


@pytest.mark.parametrize("P", [4, 2])
@pytest.mark.parametrize("R", [2, 3, 5, 8, 10])
@pytest.mark.parametrize("mode,a,b", [("semiglobal", -1, -2), ("global", -2, -2), ("fitting", -1, -1),
                                      ("overlap", -1, -3)])
def test_grouped_edges_vs_oracle(oracle, R, mode, a, b, P):
    pairs = _edge_pairs(1000 * R + 10 * P + len(mode), R, mode, P)
    res, st = _align(mode, pairs, a, b, "1", str(P))
    assert st["grouped"] > 0 and st["group_pairs"] == P and st["R"] == R, st
    check_results(oracle, mode, pairs, res, "blosum62", a, b)
    ref, _ = _align(mode, pairs, a, b, "0")
    diff = [p for p in range(len(pairs)) if _key(res[p]) != _key(ref[p])]
    assert not diff, diff[:10]


@pytest.mark.parametrize("mode,a,b", [("semiglobal", -1, -2), ("global", -2, -2)])
def test_grouped_batch_with_empty_pairs(oracle, mode, a, b):
    """Empty reads and empty references inside a grouped batch: the planner leaves them out of
    every group (their results are decided without a DP) while the grouped layout re-bases the
    trace arena; their results, and every grouped pair's, equal the ungrouped run and the oracle."""
    rng = random.Random(0xE0 + len(mode))
    ref = rand_seq(rng, 700, DNA)
    pairs = []
    for k in range(80):
        o = rng.randint(0, 550)
        pairs.append((mutate(rng, ref[o:o + 150], DNA, 0.05), ref))
        if k % 13 == 0:
            pairs.append((b"", ref))
        if k % 17 == 0:
            pairs.append((rand_seq(rng, 120, DNA), b""))
    pairs.append((b"", b""))
    res, st = _align(mode, pairs, a, b, "1")
    assert st["grouped"] > 0, st
    ref_res, st0 = _align(mode, pairs, a, b, "0")
    assert st0["grouped"] == 0, st0
    diff = [p for p in range(len(pairs)) if _key(res[p]) != _key(ref_res[p])]
    assert not diff, diff[:10]
    check_results(oracle, mode, pairs, res, "blosum62", a, b)


def test_grouping_declines_distinct_references(aligner, oracle):
    rng = random.Random(7)
    pairs = [(rand_seq(rng, 100, DNA), rand_seq(rng, 300, DNA)) for _ in range(200)]
    check_batch(aligner, oracle, "semiglobal", pairs, "blosum62", -1, -2, sample=sample_indices(200, 16, 3))
    assert aligner.stats()["grouped"] == 0


@pytest.fixture
def aligner():
    from biogarden_amd.alignment.aligner import SequenceAligner
    al = SequenceAligner(0)
    yield al
    al.close()
