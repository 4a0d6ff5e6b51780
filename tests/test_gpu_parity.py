"""Parity of the HIP path (libbiogarden_gpu.so through the C ABI) with the reference.

* the reference's own integration goldens and doctests, through the SequenceAligner mirror
  (reads like tests/integration.rs:234-312);
* seeded random pairs against the CPU oracle (oracle/refcpu.c) — bit-exact score and strings —
  over every mode, a<b / a=b / a>b, DNA / protein, edge lengths, and every kernel geometry;
* the fresh-aligner reference model: wherever the reference returns, so do we, identically;
  wherever it panics/hangs we flag it (status 3/4);
* full BASELINE size (10 kbp x 10 kbp semiglobal, blosum62 -1/-2) through size-independent
  properties, plus two full pairs against the oracle.
"""
import os
import random
import zlib

import pytest

from conftest import REF_FIX, REFERENCE_DOCTESTS, REFERENCE_GOLDENS, read_fasta

pytestmark = pytest.mark.gpu

from parity_util import DNA, PROT, check_batch, mutate, rand_seq, rescore_semiglobal


@pytest.fixture
def aligner():
    """A new SequenceAligner per test (the reference's tests each start from
    SequenceAligner::new(), whose 1024 x 1024 scratch the divergence flags depend on)."""
    from biogarden_amd.alignment.aligner import SequenceAligner
    al = SequenceAligner(0)
    yield al
    al.close()


# ------------------------------------------------------------------ reference goldens


@pytest.mark.parametrize("mode,scoring,a,b,expected", REFERENCE_GOLDENS)
def test_integration_golden(aligner, mode, scoring, a, b, expected):
    from biogarden_amd.alignment import score
    from biogarden_amd.io import fasta
    inputs = fasta.read_tile(os.path.join(REF_FIX, "input", "%s_alignment.fasta" % mode))
    outputs = fasta.read_tile(os.path.join(REF_FIX, "output", "%s_alignment.fasta" % mode))
    fn = getattr(aligner, "%s_alignment" % mode)
    align_score, s1_aligned, s2_aligned = fn(inputs[0], inputs[1], getattr(score, scoring), a, b)
    assert align_score == expected
    assert s1_aligned == outputs[0]
    assert s2_aligned == outputs[1]


@pytest.mark.parametrize("case", REFERENCE_DOCTESTS, ids=lambda c: c[0])
def test_doctest(aligner, case):
    from biogarden_amd.alignment import score
    from biogarden_amd.ds import Sequence
    mode, s1, s2, scoring, a, b, exp, e1, e2 = case
    fn = getattr(aligner, "%s_alignment" % mode)
    got = fn(Sequence(s1), Sequence(s2), getattr(score, scoring), a, b)
    assert got == (exp, Sequence(e1), Sequence(e2))


def test_errors_like_reference(aligner):
    from biogarden_amd.alignment import score
    from biogarden_amd.error import InvalidArgumentRange, InvalidInputSize, ReferencePanic
    with pytest.raises(InvalidArgumentRange):
        aligner.global_alignment(b"AC", b"AC", score.unit, 1, -1)
    with pytest.raises(InvalidArgumentRange):
        aligner.local_alignment(b"AC", b"AC", score.unit, -1, 1)
    with pytest.raises(InvalidInputSize):
        aligner.fitting_alignment(b"A", b"AC", score.unit, -1, -1)
    with pytest.raises(ReferencePanic):
        aligner.global_alignment(b"Ac", b"AC", score.unit, -1, -1)
    assert aligner.semiglobal_alignment(b"GGACGT", b"ACGTCC", score.unit, -1, -1) == (4, b"ACGT--", b"ACGTCC")


def test_custom_closure(aligner, oracle):
    """An arbitrary scoring closure is tabulated (A.8) and matches the oracle on its table."""
    def match_mismatch(x, y):
        return 3 if x == y else -2
    s1, s2 = b"ACGTTGCAACG", b"ACGTGCATACG"
    got = aligner.global_alignment(s1, s2, match_mismatch, -4, -1)
    sc = oracle.scoring(match_mismatch)
    st, score, o1, o2 = oracle.align("global", s1, s2, sc, -4, -1, exact=True)
    assert st == 0 and got == (score, o1, o2)


@pytest.mark.parametrize("mode,a,b", [("global", -11, -1), ("local", -11, -1),
                                      ("semiglobal", -3, -3), ("overlap", -4, -2)])
def test_custom_closure_wide_alphabet(aligner, oracle, mode, a, b):
    """A closure over more than 32 distinct bytes (the reference's &dyn Fn(&u8, &u8) -> i32
    takes any): tabulated as a k x k table (bg_batch_prepare_table), bit-exact with the oracle
    on the same table."""
    rng = random.Random(len(mode) * 31 - a * 7 - b)
    alpha = bytes(range(48, 48 + 70))

    def fn(x, y):
        return 5 if x == y else (-2 if (x ^ y) & 1 else -4)
    pairs = []
    for n1, n2 in ((200, 180), (700, 1300), (65, 64), (1, 7), (2000, 1900)):
        s1 = rand_seq(rng, n1, alpha)
        pairs.append((s1, mutate(rng, s1, alpha, 0.15)[:n2]))
    res = aligner.align_batch(mode, pairs, fn, a, b)
    sc = oracle.wide_scoring(fn, alpha)
    for (s1, s2), r in zip(pairs, res):
        st, score, o1, o2 = oracle.align(mode, s1, s2, sc, a, b, exact=True)
        assert st == 0 and r.status in (0, 4) and tuple(r[:3]) == (score, o1, o2), (mode, len(s1), len(s2))
    assert aligner.stats()["checkpoint"] == 1 and aligner.stats()["tagged"] == 0


@pytest.mark.parametrize("mode,a,b", [("global", -20000, -3000), ("local", -15000, -15000),
                                      ("semiglobal", -9000, -12000), ("fitting", -100, -40000)])
def test_custom_closure_beyond_int16(aligner, oracle, mode, a, b):
    """Scores whose S - a leave int16 (the reference's closure is any i32): the mask-trace
    kernel with int32 profile entries, which keeps the reference's wrapping i32 arithmetic."""
    rng = random.Random(len(mode) + a)

    def big(x, y):
        return 30000 if x == y else -25000 - 7 * abs(x - y)
    pairs = []
    for n1, n2 in ((150, 140), (600, 900), (64, 65), (1, 3), (1300, 1200)):
        s1 = rand_seq(rng, n1, PROT)
        pairs.append((s1, mutate(rng, s1, PROT, 0.2)[:n2]))
    res = aligner.align_batch(mode, pairs, big, a, b)
    sc = oracle.scoring(big)
    for (s1, s2), r in zip(pairs, res):
        st, score, o1, o2 = oracle.align(mode, s1, s2, sc, a, b, exact=True)
        if st != 0:
            assert r.status == st or r.status == 4
            continue
        assert r.status in (0, 4) and tuple(r[:3]) == (score, o1, o2), (mode, len(s1), len(s2))
    st = aligner.stats()
    assert st["checkpoint"] == 0 and st["tagged"] == 0 and st["R"] == 4, st


@pytest.mark.parametrize("mode,a,b,nsym,big", [("global", -11, -1, 70, 900), ("local", -300, -300, 70, 900),
                                                ("semiglobal", -5, -9, 200, 900), ("fitting", -40, -3, 256, 900),
                                                ("overlap", -4, -6, 90, 40000), ("global", -30000, -2, 120, 40000),
                                                # K x 64 int32 profiles beyond the LDS: tables in HBM
                                                ("global", -11, -1, 256, 40000), ("local", -300, -300, 200, 40000),
                                                ("semiglobal", -5, -9, 160, 40000)])
def test_wide_alphabet_beyond_int8(aligner, oracle, mode, a, b, nsym, big):
    """More than 32 symbols with scores the score-only int8 kernels cannot take (the reference's
    closure is any i32 over any bytes, score.rs:38-41): the mask-trace kernel, its k x k table
    read from HBM (int16 entries, or int32 when S - a leaves int16; beyond ~150 int32 codes the
    per-wave profiles live in HBM too, where BG_E_ALPHABET used to refuse), bit-exact with the
    oracle."""
    rng = random.Random(nsym * 7 + big - a)
    alpha = bytes(range(256 - nsym, 256))

    def fn(x, y):
        return big if x == y else -(big // 3) - 3 * ((x * 7 + y) % 11)
    pairs = []
    # 3000 rows: 12 strips at R = 4, through HBM boundary rows when one wave fills the LDS
    for n1, n2 in ((180, 170), (600, 900), (64, 65), (1, 9), (1300, 1200), (3000, 2800)):
        s1 = rand_seq(rng, n1, alpha)
        s2 = mutate(rng, s1, alpha, 0.2)[:n2]
        if mode == "fitting" and len(s2) > len(s1):
            s2 = s2[:len(s1)]
        pairs.append((s1, s2))
    res = aligner.align_batch(mode, pairs, fn, a, b)
    sc = oracle.wide_scoring(fn, alpha)
    matched = 0
    for (s1, s2), r in zip(pairs, res):
        st, score, o1, o2 = oracle.align(mode, s1, s2, sc, a, b, exact=True)
        if st != 0:                      # the reference panics (traceback underflow): so do we
            assert r.status == st, (mode, len(s1), len(s2), st, r.status)
            continue
        assert r.status in (0, 4) and tuple(r[:3]) == (score, o1, o2), (mode, len(s1), len(s2))
        matched += 1
    assert matched >= 2
    st = aligner.stats()
    assert st["checkpoint"] == 0 and st["tagged"] == 0 and st["R"] == 4, st


def test_closure_panics_only_where_reached(aligner, oracle):
    """A closure that panics on one (byte1, byte2) makes exactly the pairs whose DP evaluates
    it unscorable (status 3); the other pairs of the batch align normally (A.8)."""
    from biogarden_amd.error import ReferencePanic

    def total(x, y):
        return 3 if x == y else -2

    def partial(x, y):
        if (x, y) == (ord("A"), ord("T")):
            raise IndexError("score table index out of range")
        return total(x, y)

    pairs = [(b"ACGGA", b"GTTAC"), (b"CCGCG", b"GTAGG"), (b"TTATA", b"CCGCA")]
    res = aligner.align_batch("global", pairs, partial, -4, -1)
    assert [r.status for r in res] == [3, 0, 0]
    sc = oracle.scoring(total)
    for (s1, s2), r in list(zip(pairs, res))[1:]:
        st, score, o1, o2 = oracle.align("global", s1, s2, sc, -4, -1, exact=True)
        assert st == 0 and tuple(r[:3]) == (score, o1, o2)
    with pytest.raises(ReferencePanic):
        aligner.global_alignment(b"ACGGA", b"GTTAC", partial, -4, -1)


# ------------------------------------------------------------------ seeded random vs oracle

GAPS = [(-11, -1), (-2, -2), (-1, -2), (-3, -1), (0, 0), (-5, -5)]


@pytest.mark.parametrize("mode", ["global", "local", "fitting", "overlap", "semiglobal"])
@pytest.mark.parametrize("alpha,scoring", [(DNA, "blosum62"), (DNA, "unit"), (PROT, "blosum62"), (PROT, "pam250")])
def test_random_small(aligner, oracle, mode, alpha, scoring):
    rng = random.Random(zlib.crc32(repr((mode, alpha, scoring)).encode()))   # stable across runs
    lens = [0, 1, 2, 3, 7, 31, 63, 64, 65, 100, 127, 128, 129, 200, 255, 256, 257, 300]
    for a, b in GAPS:
        pairs = []
        for _ in range(24):
            n1, n2 = rng.choice(lens), rng.choice(lens)
            if mode == "fitting" and n1 < n2 and rng.random() < 0.8:
                n1, n2 = n2, n1
            s1 = rand_seq(rng, n1, alpha)
            s2 = mutate(rng, s1, alpha)[:n2] if rng.random() < 0.5 else rand_seq(rng, n2, alpha)
            pairs.append((s1, s2))
        check_batch(aligner, oracle, mode, pairs, scoring, a, b)


@pytest.mark.parametrize("R,W", [(4, 1), (4, 3), (8, 1), (8, 2), (8, 4), (8, 16)])
@pytest.mark.parametrize("mode,a,b", [("semiglobal", -1, -2), ("local", -11, -1), ("global", -11, -1), ("overlap", -2, -2)])
def test_geometries_multistrip(aligner, oracle, R, W, mode, a, b):
    """Pairs spanning several strips, every pipelining depth; DNA and protein."""
    rng = random.Random(R * 100 + W + len(mode))
    aligner.set_tuning(R, W)
    try:
        for alpha, scoring in ((DNA, "blosum62"), (PROT, "blosum62")):
            pairs = []
            for n1, n2 in ((1500, 1400), (700, 2100), (513, 64), (2049, 511), (64 * R * 3, 333), (1, 900)):
                s1 = rand_seq(rng, n1, alpha)
                s2 = mutate(rng, s1, alpha, 0.15)[:n2]
                pairs.append((s1, s2))
            check_batch(aligner, oracle, mode, pairs, scoring, a, b, fresh=False)
    finally:
        aligner.set_tuning(0, 0)


@pytest.mark.parametrize("kernel", ["checkpoint", "tagged", "mask"])
@pytest.mark.parametrize("R,W", [(2, 4), (3, 16), (4, 3), (5, 1), (5, 8), (8, 16), (10, 2), (10, 16)])
@pytest.mark.parametrize("mode", ["semiglobal", "local", "overlap", "fitting", "global"])
def test_geometries_linear_dna(aligner, oracle, R, W, mode, kernel):
    """The metric-path kernels (linear gaps a >= b, DNA register profile) at every strip height:
    score-only DP + checkpoint traceback, tagged DP with the full trace, mask-trace DP."""
    rng = random.Random(R * 1000 + W)
    aligner._h.set_kernel_options(kernel != "mask", kernel == "checkpoint", kernel != "mask")
    aligner.set_tuning(R, W)
    try:
        pairs = []
        for n1, n2 in ((1500, 1400), (700, 2100), (64 * R * 3 + 1, 333), (640, 640), (2, 5), (2100, 2100)):
            s1 = rand_seq(rng, n1, DNA)
            s2 = mutate(rng, s1, DNA, 0.15)[:n2]
            pairs.append((s1, s2))
        check_batch(aligner, oracle, mode, pairs, "blosum62", -1, -2, fresh=False)
        st = aligner.stats()
        if mode != "local":
            assert st["checkpoint"] == (kernel == "checkpoint") and st["tagged"] == (kernel != "mask"), st
    finally:
        aligner.set_tuning(0, 0)
        aligner._h.set_kernel_options(True)


@pytest.mark.parametrize("kernel", ["affine_checkpoint", "mask"])
@pytest.mark.parametrize("R,W", [(2, 1), (2, 16), (4, 3), (4, 8), (8, 2), (8, 5)])
@pytest.mark.parametrize("mode,a,b", [("local", -11, -1), ("global", -11, -1), ("semiglobal", -3, -1),
                                      ("overlap", -5, -2), ("fitting", -4, -1), ("local", -2, -2),
                                      ("global", -1, -2)])
def test_geometries_affine(aligner, oracle, R, W, mode, a, b, kernel):
    """The affine / local / protein path at every strip height: score-only DP with per-chunk
    checkpoints + traceback recomputing full 4-bit-trace chunks, against the mask-trace kernel;
    DNA and protein, pairs spanning several strips and the LDS mailbox / HBM round wraps."""
    rng = random.Random(R * 1000 + W + a * 7 + b)
    aligner._h.set_kernel_options(True, True, kernel == "affine_checkpoint")
    aligner.set_tuning(R, W)
    try:
        for alpha, scoring in ((DNA, "blosum62"), (PROT, "blosum62")):
            pairs = []
            for n1, n2 in ((1500, 1400), (700, 2100), (64 * R * 3 + 1, 333), (640, 640), (2, 5),
                           (2100, 1900), (65, 1), (1, 70)):
                if mode == "fitting" and n1 < n2:
                    n1, n2 = n2, n1
                s1 = rand_seq(rng, n1, alpha)
                s2 = mutate(rng, s1, alpha, 0.15)[:n2]
                pairs.append((s1, s2))
            check_batch(aligner, oracle, mode, pairs, scoring, a, b, fresh=False)
            st = aligner.stats()
            if not (a >= b and mode != "local" and alpha == DNA):
                assert st["checkpoint"] == (kernel == "affine_checkpoint") and st["tagged"] == 0, st
    finally:
        aligner.set_tuning(0, 0)
        aligner._h.set_kernel_options(True)


@pytest.mark.parametrize("ckpt", [True, False])
@pytest.mark.parametrize("R", [0, 2, 5])
@pytest.mark.parametrize("mode", ["semiglobal", "global", "overlap", "fitting"])
def test_wide_pairs(aligner, oracle, mode, R, ckpt):
    """Few long pairs: the tagged kernel spreads each pair's strips over a group of workgroups
    (global agent-scope progress counters, groups spanning XCDs); bit-exact against the oracle."""
    rng = random.Random(31 + R)
    aligner.set_tuning(R, 0)
    aligner._h.set_kernel_options(True, ckpt)
    try:
        pairs = []
        for n1, n2 in ((5000, 4100), (4500, 3000), (4103, 900), (300, 200), (6000, 64)):
            s1 = rand_seq(rng, n1, DNA)
            s2 = mutate(rng, s1, DNA, 0.1)[:n2]
            pairs.append((s1, s2))
        res = check_batch(aligner, oracle, mode, pairs, "blosum62", -1, -2, fresh=False)
        st = aligner.stats()
        assert st["tagged"] == 1 and st["wide"] == 1 and st["workgroups"] > len(pairs), st
        assert st["checkpoint"] == int(ckpt)
        assert all(r.status == 0 for r in res)
    finally:
        aligner.set_tuning(0, 0)
        aligner._h.set_kernel_options(True)


def test_buffer_edge_and_divergence(aligner, oracle):
    """Lengths around the reference's 1024x1024 default scratch (A.7)."""
    rng = random.Random(7)
    for mode, a, b in (("global", -11, -1), ("semiglobal", -1, -1), ("overlap", -2, -2),
                       ("fitting", -1, -1), ("local", -11, -1)):
        pairs = []
        for n1, n2 in ((1024, 10), (10, 1024), (1023, 1023), (1025, 17), (0, 1024), (1024, 0), (1024, 1024)):
            pairs.append((rand_seq(rng, n1, DNA), rand_seq(rng, n2, DNA)))
        check_batch(aligner, oracle, mode, pairs, "unit", a, b)


def test_unscorable_and_empty(aligner, oracle):
    pairs = [(b"ACGT", b"ACXT"), (b"acgt", b"ACGT"), (b"", b"ACGT"), (b"ACGT", b""), (b"", b""),
             (b"A-C", b"AC")]
    for mode in ("global", "local", "semiglobal", "overlap"):
        check_batch(aligner, oracle, mode, pairs, "blosum62", -3, -1)


# ------------------------------------------------------------------ BASELINE-size properties


def test_baseline_size_semiglobal_properties(aligner, oracle):
    from biogarden_amd.alignment import score
    rng = random.Random(0xB10A11F0)
    pairs = []
    for p in range(8):
        s1 = rand_seq(rng, 10000, DNA)
        s2 = mutate(rng, s1, DNA, 0.2)[:10000] if p % 2 else rand_seq(rng, 10000, DNA)
        pairs.append((s1, s2))
    res = aligner.align_batch("semiglobal", pairs, score.blosum62, -1, -2)
    table = score.blosum62.table()
    for (s1, s2), r in zip(pairs, res):
        assert r.status == 0
        sc, d1, d2 = rescore_semiglobal(r, s1, s2, table, -1)
        assert sc == r[0]
        assert len(r[1]) == len(r[2])
        assert d1 == s1[r.start[0] if r.end[0] == len(s1) else 0:]
        assert s2.endswith(d2)
    # two full pairs bit-exact against the oracle (1e8 cells each)
    for (s1, s2), r in list(zip(pairs, res))[:2]:
        st, sc, o1, o2 = oracle.align("semiglobal", s1, s2, "blosum62", -1, -2, exact=True)
        assert (st, sc, o1, o2) == (0, r[0], bytes(r[1].chain), bytes(r[2].chain))


def test_deterministic(aligner):
    from biogarden_amd.alignment import score
    rng = random.Random(3)
    pairs = [(rand_seq(rng, 3000, DNA), rand_seq(rng, 2500, DNA)) for _ in range(4)]
    r1 = aligner.align_batch("local", pairs, score.blosum62, -11, -1)
    r2 = aligner.align_batch("local", pairs, score.blosum62, -11, -1)
    assert [(x[0], x[1], x[2]) for x in r1] == [(x[0], x[1], x[2]) for x in r2]


def test_pipelined_executes_match_single():
    """Depth-2 pipeline (traceback of execute k overlapping DP of k+1) returns what a single
    serialised execute returns."""
    from biogarden_amd import _native
    rng = random.Random(11)
    pairs = [(rand_seq(rng, 2500, DNA), rand_seq(rng, 2200, DNA)) for _ in range(6)]
    sc = _native.builtin_scoring(_native.BG_BLOSUM62)
    h = _native.Handle(0)
    h.set_pipeline(1)
    want = h.align_batch("semiglobal", pairs, sc, -1, -2)
    h.set_pipeline(2)
    h.prepare("semiglobal", pairs, sc, -1, -2)
    for _ in range(5):
        h.execute()
    got = h.fetch()
    h.close()
    assert got == want


# ------------------------------------------------------------------ asynchronous recomputation
def _long_gap_pairs(rng):
    """Paths that stress the traceback's chunk cache: a 3000-column insertion (the walk crosses
    ~47 chunks of one strip: direct-mapped table collisions 16 chunks apart), a 2500-row deletion
    (the walk climbs strips in one chunk column), and a diagonal pair for the prediction."""
    base = rand_seq(rng, 6000, DNA)
    ins = base[:3000] + rand_seq(rng, 3000, DNA) + base[3000:]
    dele = base[:1500] + base[4000:]
    return [(base, ins), (base, dele), (base, mutate(rng, base, DNA, 0.15))]


@pytest.mark.parametrize("mode,a,b", [("semiglobal", -1, -2), ("global", -2, -2), ("overlap", -1, -1)])
def test_traceback_async_matches_barriers_and_oracle(aligner, oracle, mode, a, b):
    """The helper-wave recomputation (default) and the barrier form (bg_set_option fin_sync = 1) give the
    oracle's strings on long-gap paths, at the metric geometry and at a short-strip one."""
    from biogarden_amd.alignment import score
    rng = random.Random(0xA5C)
    pairs = _long_gap_pairs(rng)
    expect = [oracle.align(mode, s1, s2, "blosum62", a, b, exact=True) for s1, s2 in pairs]
    try:
        for R, W in ((8, 16), (2, 4)):
            aligner.set_tuning(R, W)
            for sync in (False, True):
                aligner.set_option("fin_sync", 1 if sync else None)
                res = aligner.align_batch(mode, pairs, score.blosum62, a, b)
                for e, r in zip(expect, res):
                    assert r.status in (0, 4), (R, W, sync, r.status)
                    assert (e[1], e[2], e[3]) == (r[0], bytes(r[1].chain), bytes(r[2].chain)), (R, W, sync)
    finally:
        aligner.set_option("fin_sync", None)
        aligner.set_tuning(0, 0)
