"""GPU parity at BASELINE.json's configurations, at their real shapes and
through the default planner, so the geometry each config actually runs is the one tested:

* C1  semiglobal on the reference's test FASTA, blosum62 -1/-2 (examples/from_file.rs:14-31)
      against the oracle-derived golden (tests/golden/derived/, labelled derived);
* C2  1024 x (1000 x 1000) local DNA, -11/-1 — many pairs: the 2-wave / 3-slot traceback;
* C3  100 kbp x 100 kbp semiglobal (WIDE): full-size properties + a 20 kbp WIDE pair bit-exact;
* C4  a 1024-pair slice of 150 bp reads vs 10 kbp refs, semiglobal -1/-2 (row branch, R = 3);
* C5  one GPU's 4080-pair share of the 256-protein all-vs-all, global -11/-1;
* MA  the metric's shape with a genuinely affine gap model (-11/-1, open < extend);
plus the reference behaviours the configs do not reach: positive gap penalties (semiglobal /
overlap accept them, aligner.rs:290-360), the reused aligner's scratch history (aligner.rs:92-94),
pairs beyond the checkpoint tracebacks' chunk keys, and the traceback's forward-progress path.

Score and both aligned strings are compared bit-exactly with oracle.align(..., exact=True) on
a seeded sample of each batch (every pair for the small ones).
"""
import json
import os
import random

import pytest

from conftest import GOLDEN, REF_FIX, read_fasta
from parity_util import DNA, check_batch, mutate, rand_seq, rescore_semiglobal, sample_indices

pytestmark = pytest.mark.gpu


@pytest.fixture
def aligner():
    from biogarden_amd.alignment.aligner import SequenceAligner
    al = SequenceAligner(0)
    yield al
    al.close()


def _w():
    from tools import workloads
    return workloads


# ------------------------------------------------------------------ C1


def test_C1_from_file_derived_golden(aligner):
    """examples/from_file.rs: semiglobal_alignment of the two records with blosum62, -1, -2."""
    from biogarden_amd.alignment import score
    from biogarden_amd.io import fasta
    with open(os.path.join(GOLDEN, "derived", "C1_semiglobal_blosum62_o1_e2.json")) as f:
        gold = json.load(f)
    assert gold["derived"] is True
    tile = fasta.read_tile(os.path.join(REF_FIX, "input", "semiglobal_alignment.fasta"))
    got = aligner.semiglobal_alignment(tile[0], tile[1], score.blosum62, -1, -2)
    assert got[0] == gold["score"]
    assert bytes(got[1].chain) == gold["aligned1"].encode()
    assert bytes(got[2].chain) == gold["aligned2"].encode()
    st = aligner.stats()
    assert st["tagged"] == 1 and st["checkpoint"] == 1, st


# ------------------------------------------------------------------ C2, C4, C5: many pairs


def test_C2_1024_local_dna_full_batch(aligner, oracle):
    w = _w()
    pairs = w.c2_pairs()
    res = check_batch(aligner, oracle, "local", pairs, "blosum62", -11, -1,
                      sample=sample_indices(len(pairs), 32, 2))
    st = aligner.stats()
    # the affine / local checkpoint path with the many-pair local finish geometry (fin_geom)
    assert st["checkpoint"] == 1 and st["local"] == 1 and st["tagged"] == 0, st
    assert (st["fin_waves"], st["fin_slots"]) == (1, 2), st   # local: one wave, two slots
    assert st["npairs"] == 1024
    assert all(r.status == 0 for r in res)


def test_C4_reads_vs_refs_slice(aligner, oracle):
    w = _w()
    pairs = w.c4_pairs(nrefs=8, reads_per_ref=128)
    res = check_batch(aligner, oracle, "semiglobal", pairs, "blosum62", -1, -2,
                      sample=sample_indices(len(pairs), 48, 4))
    st = aligner.stats()
    assert st["tagged"] == 1 and st["checkpoint"] == 1 and st["wide"] == 0, st
    # four reads of one reference per wave (bg_grp_kernel.hip), the walker recomputing alone
    assert st["grouped"] == 8 * 32 and st["group_pairs"] == 4 and st["R"] == 10, st
    assert (st["fin_waves"], st["fin_slots"]) == (1, 6), st
    assert all(r.status == 0 for r in res)
    # 150 bp reads against 10 kbp refs: the row branch (end cell in the last row)
    assert all(r.end[0] == 150 for r in res)


def test_C4_rank0_share_as_benched(aligner, oracle):
    """The 8 192-pair share the bench times (rank 0's LPT shard of the 65 536-read job over 8
    GPUs, tools/configs.py C4): the grouped plan at full size, 48 sampled pairs string-exact."""
    from biogarden_amd.shard import lpt_shards
    w = _w()
    allp = w.c4_pairs()
    share = lpt_shards([(len(x), len(y)) for x, y in allp], 8)[0]
    pairs = [allp[p] for p in share]
    assert len(pairs) == 8192
    res = check_batch(aligner, oracle, "semiglobal", pairs, "blosum62", -1, -2,
                      sample=sample_indices(len(pairs), 48, 6))
    st = aligner.stats()
    assert st["tagged"] == 1 and st["checkpoint"] == 1 and st["group_pairs"] == 4 and st["R"] == 10, st
    assert st["grouped"] == 2048, st
    assert all(r.status == 0 and r.end[0] == 150 for r in res)


def test_C5_protein_all_vs_all_share(aligner, oracle):
    w = _w()
    pairs = w.c5_pairs(rank=0, world=8)
    assert len(pairs) == 4080
    res = check_batch(aligner, oracle, "global", pairs, "blosum62", -11, -1,
                      sample=sample_indices(len(pairs), 32, 5))
    st = aligner.stats()
    assert st["checkpoint"] == 1 and st["tagged"] == 0 and st["dna"] == 0, st
    assert (st["fin_waves"], st["fin_slots"]) == (2, 3), st
    assert all(r.status == 0 for r in res)


# ------------------------------------------------------------------ C3: one long pair (WIDE)


def test_C3_100k_semiglobal_full_size_properties(aligner):
    """10^10 cells: the oracle cannot run it; size-independent properties instead — the
    emitted alignment rescored under the linear model (a >= b) equals the score, de-gapping
    gives back the consumed residues, the end cell follows the semiglobal rule's shape."""
    from biogarden_amd.alignment import score
    w = _w()
    (s1, s2), = w.c3_pair()
    r, = aligner.align_batch("semiglobal", [(s1, s2)], score.blosum62, -1, -2)
    st = aligner.stats()
    assert st["wide"] == 1 and st["tagged"] == 1, st
    assert r.status == 0
    sc, d1, d2 = rescore_semiglobal(r, s1, s2, score.blosum62.table(), -1)
    assert sc == r[0]
    assert len(r[1]) == len(r[2])
    colcase = r.end[0] < len(s1)
    assert (r.end[1] == len(s2)) if colcase else (r.end[0] == len(s1))
    assert d1 == (s1 if colcase else s1[r.start[0]:])
    assert d2 == (s2[r.start[1]:] if colcase else s2)
    assert r[0] > 0


def test_C3_wide_20k_string_parity(aligner, oracle):
    from tools import workloads as w
    rng = w.rng_for("C3", salt=17)
    s1 = w.rand_seq(rng, w.DNA, 20000)
    s2 = w.rand_seq(rng, w.DNA, 20000)
    res = check_batch(aligner, oracle, "semiglobal", [(s1, s2)], "blosum62", -1, -2)
    st = aligner.stats()
    assert st["wide"] == 1 and st["workgroups"] > 1, st
    assert res[0].status == 0


# ------------------------------------------------------------------ M: the metric's own batch


def test_M_metric_batch_at_bench_geometry(aligner, oracle):
    """bench.py's metric batch exactly (256 x 10 kbp x 10 kbp uniform DNA, semiglobal blosum62
    -1/-2, rank 0's seed) through the default planner, which must pick the bench's geometry
    (R = 8, W = 16, checkpoint traceback with 4-wave finish workgroups); score and both strings of
    five pairs spread over the LPT order against the oracle, every status 0."""
    w = _w()
    pairs = w.metric_pairs(256)          # = bench.make_pairs(256, 10000, 10000, SEED) at rank 0
    res = check_batch(aligner, oracle, "semiglobal", pairs, "blosum62", -1, -2,
                      sample=[0, 63, 128, 200, 255])
    st = aligner.stats()
    assert (st["R"], st["waves"], st["tagged"], st["checkpoint"], st["wide"]) == (8, 16, 1, 1, 0), st
    assert (st["fin_waves"], st["fin_slots"]) == (4, 0), st
    assert all(r.status == 0 for r in res)


# ------------------------------------------------------------------ MA: a < b at the metric shape


def test_MA_metric_shape_affine_gaps(aligner, oracle):
    """256 x 10 kbp x 10 kbp semiglobal, blosum62 -11/-1 (open < extend: the real Gotoh DP with
    the reference's one-cell-late X/Y traceback); two pairs against the oracle."""
    w = _w()
    pairs = w.metric_pairs(256, seed=w.SEED0 + 6)
    res = check_batch(aligner, oracle, "semiglobal", pairs, "blosum62", -11, -1,
                      sample=[0, 255])
    st = aligner.stats()
    assert st["affine"] == 1 and st["checkpoint"] == 1 and st["tagged"] == 0, st
    assert all(r.status == 0 for r in res)


# ------------------------------------------------------------------ positive gap penalties


@pytest.mark.parametrize("mode", ["semiglobal", "overlap"])
@pytest.mark.parametrize("a,b", [(1, 1), (2, 1), (1, 2), (0, 3), (3, 0)])
@pytest.mark.parametrize("alpha,scoring", [(DNA, "blosum62"), (DNA, "unit"),
                                           (b"ACDEFGHIKLMNPQRSTVWY", "blosum62")])
def test_positive_gaps(aligner, oracle, mode, a, b, alpha, scoring):
    """semiglobal / overlap do no sign check (aligner.rs:290-360): positive penalties reach the
    DP.  Linear (a >= b) and affine (a < b) frames both, against the exact-size oracle."""
    rng = random.Random(a * 31 + b * 7 + len(mode) + len(alpha))
    pairs = []
    for n1, n2 in ((300, 280), (700, 1500), (64, 65), (1, 9), (2100, 1900), (129, 0)):
        s1 = rand_seq(rng, n1, alpha)
        s2 = mutate(rng, s1, alpha, 0.2)[:n2] if rng.random() < 0.5 else rand_seq(rng, n2, alpha)
        pairs.append((s1, s2))
    check_batch(aligner, oracle, mode, pairs, scoring, a, b)


# ------------------------------------------------------------------ reused aligner


def test_reused_aligner_scratch_history(oracle):
    """One SequenceAligner reused across calls, as the reference's is: its scratch grows to
    (len1+1, len2+1) only on a strict overflow (aligner.rs:92-94) and both dims are reset, so a
    later pair of length L+1 panics it and a length-1024 pair after a 2000 x 2000 call does not.
    Compared with one reference-faithful oracle aligner replayed in the same order."""
    from biogarden_amd.alignment import score
    from biogarden_amd.alignment.aligner import SequenceAligner
    rng = random.Random(99)
    seqs = lambda n: rand_seq(rng, n, DNA)  # noqa: E731
    calls = [("global", 2000, 2000), ("global", 1024, 1024), ("semiglobal", 1500, 700),
             ("global", 1501, 300), ("global", 1500, 300), ("local", 1024, 1024),
             ("global", 300, 701), ("overlap", 10, 20), ("semiglobal", 5, 5), ("fitting", 30, 20),
             ("local", 2001, 50), ("global", 2001, 50), ("global", 2002, 51)]
    al = SequenceAligner(0)
    ref = oracle.Aligner(exact=False)
    try:
        assert al.buffer_size == ref.buffer_size() == (1024, 1024)
        for mode, n1, n2 in calls:
            s1 = seqs(n1)
            s2 = mutate(rng, s1, DNA, 0.1)[:n2] if n2 <= n1 else seqs(n2)
            r, = al.align_batch(mode, [(s1, s2)], score.unit, -1, -1)
            fst, fsc, f1, f2 = ref.align(mode, s1, s2, "unit", -1, -1)
            est, esc, e1, e2 = oracle.align(mode, s1, s2, "unit", -1, -1, exact=True)
            assert al.buffer_size == ref.buffer_size(), (mode, n1, n2)
            if fst == 0 and (fsc, f1, f2) == (esc, e1, e2):
                assert r.status == 0 and (r[0], bytes(r[1].chain), bytes(r[2].chain)) == (fsc, f1, f2), \
                    (mode, n1, n2, r.status)
            else:
                assert r.status == 4, (mode, n1, n2, fst, r.status)   # panics / stale answer
                assert (r[0], bytes(r[1].chain), bytes(r[2].chain)) == (esc, e1, e2)
    finally:
        al.close()


# ------------------------------------------------------------------ size limits of the checkpoints


@pytest.mark.parametrize("mode,a,b,n1,n2", [("local", -11, -1, 530000, 100),
                                            ("semiglobal", -1, -2, 530000, 100),
                                            ("semiglobal", -1, -2, 64, 4200000)])
def test_beyond_checkpoint_chunk_keys(aligner, oracle, mode, a, b, n1, n2):
    """Pairs with >= 4096 strips (n1 = 530k at R = 2) or >= 65536 chunks (n2 = 4.2M) do not fit
    the checkpoint tracebacks' 32-bit chunk keys; the host routes them to the full-trace kernels.
    Bit-exact against the oracle."""
    from tools import workloads as w
    rng = w.rng_for("C3", salt=n1 + n2)
    s1 = w.rand_seq(rng, w.DNA, n1)
    s2 = w.rand_seq(rng, w.DNA, n2)
    aligner.set_tuning(2, 0)
    try:
        res = check_batch(aligner, oracle, mode, [(s1, s2)], "blosum62", a, b, fresh=False)
    finally:
        aligner.set_tuning(0, 0)
    st = aligner.stats()
    assert st["checkpoint"] == 0, st
    assert res[0].status == 0


# ------------------------------------------------------------------ traceback forward progress


@pytest.mark.parametrize("slots", ["5", "6"])
def test_traceback_walker_self_service(aligner, oracle, slots):
    """BG_FIN_SELFSERVE: the walker recomputes every missed chunk itself instead of waiting for
    a helper (the path that guarantees forward progress when every helper is busy); with the
    fewest slots the asynchronous form allows.  Same strings as the oracle, every status 0 (a
    walker evicting a chunk it needs next would thrash into BG_INTERNAL)."""
    from biogarden_amd.alignment import score
    rng = random.Random(0x5E1F)
    base = rand_seq(rng, 6000, DNA)
    # the last two walk (near-)diagonally from (6000, 6000): across every strip boundary at a
    # chunk corner, where the walker's 2 x 2 chunk footprint matters for its own evictions
    pairs = [(base, base[:3000] + rand_seq(rng, 3000, DNA) + base[3000:]),
             (base, base[:1500] + base[4000:]), (base, mutate(rng, base, DNA, 0.15)),
             (base, base), (base, mutate(rng, base, DNA, 0.01))]
    expect = [oracle.align("semiglobal", s1, s2, "blosum62", -1, -2, exact=True) for s1, s2 in pairs]
    try:
        with aligner.options(fin_selfserve=1, fin_slots=int(slots)):
            for R, W in ((8, 16), (2, 4)):
                aligner.set_tuning(R, W)
                res = aligner.align_batch("semiglobal", pairs, score.blosum62, -1, -2)
                assert aligner._h.wait_diag() is None, (R, W, aligner._h.wait_diag())
                for e, r in zip(expect, res):
                    assert r.status in (0, 4), (R, W, r.status)
                    assert (e[1], e[2], e[3]) == (r[0], bytes(r[1].chain), bytes(r[2].chain)), (R, W)
    finally:
        aligner.set_tuning(0, 0)
