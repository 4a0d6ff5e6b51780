"""GPU parity of the split traceback: a few long pairs (the WIDE planner's
batches, C3's shape) walk their traceback strip by strip in parallel, from the entry columns the
exit pass and the chain give every strip, and the tail stitches the strip walks
(bg_split.hip, bg_finish_kernel's BG_PH_* phases).  Reference: backtrack and the semiglobal
assembly, src/alignment/aligner.rs:383-435 and :511-592.

Every case compares score and both strings with the oracle (oracle.align(..., exact=True)) and,
through bg_split_stats, checks that the stitched strip walks covered the whole traceback (the
tail walked no move itself), so a wrong exit map cannot hide behind the tail's sequential
fallback."""
import random

import pytest

from parity_util import DNA, mutate, rand_seq

pytestmark = pytest.mark.gpu


def _pairs(rng, shapes, rate=0.15):
    out = []
    for n1, n2 in shapes:
        s1 = rand_seq(rng, n1, DNA)
        s2 = (mutate(rng, s1, DNA, rate) * 3)[:n2] if n2 > 8 else rand_seq(rng, n2, DNA)
        out.append((s1, s2))
    return out


def _run(pairs, mode, a, b, R=0, scoring=None, opts=None, executes=1, diag=None):
    from biogarden_amd import _native
    h = _native.Handle(0)
    try:
        for k, v in (opts or {}).items():
            h.set_option(k, v)
        if R:
            h.set_tuning(R, 0)
        sc = scoring or _native.builtin_scoring(_native.BG_BLOSUM62)
        h.prepare(mode, pairs, sc, a, b)
        for _ in range(executes):
            h.execute()
        got = h.fetch()
        if diag is not None:
            diag.update(h.conc_diag())
        return got, h.stats(), h.split_stats()
    finally:
        h.close()


def _check(oracle, mode, pairs, got, a, b, scoring="blosum62"):
    for (s1, s2), r in zip(pairs, got):
        st, sc, o1, o2 = oracle.align(mode, s1, s2, scoring, a, b, exact=True)
        if st in (4, 5):
            assert r["status"] == 4, (mode, len(s1), len(s2))
            continue
        assert st == 0 and r["status"] in (0, 4), (mode, len(s1), len(s2), st, r["status"])
        assert (r["score"], r["aligned1"], r["aligned2"]) == (sc, o1, o2), (mode, len(s1), len(s2))


@pytest.mark.parametrize("R", [2, 5, 8])
@pytest.mark.parametrize("mode,a,b", [("semiglobal", -1, -2), ("global", -1, -2), ("fitting", -2, -2),
                                      ("overlap", -1, -3)])
def test_split_modes(oracle, R, mode, a, b):
    rng = random.Random(R * 17 + len(mode) * 5 - a)
    shapes = [(9000, 8700), (12000, 3000), (4200, 9500), (5000, 5100), (700, 600)]
    if mode == "fitting":
        shapes = [(n1, min(n1, n2)) for n1, n2 in shapes]
    pairs = _pairs(rng, shapes)
    got, st, sp = _run(pairs, mode, a, b, R=R)
    _check(oracle, mode, pairs, got, a, b)
    assert st["wide"] == 1 and st["split"] == 1 and st["R"] == R, st
    assert sp["pairs_overflow"] == 0 and sp["strips_taken"] > 0 and sp["tail_moves"] == 0, sp


@pytest.mark.parametrize("segc", ["1", "3", "1000"])
def test_split_segment_lengths(oracle, monkeypatch, segc):
    """Exit-pass segments of 1, 3 and 1000 chunks: the symbolic exits are resolved across every
    segment boundary of a strip (1), at odd positions (3), or never arise (one segment)."""
    rng = random.Random(int(segc))
    pairs = _pairs(rng, [(9000, 9100), (6000, 2500)], rate=0.25)
    got, st, sp = _run(pairs, "semiglobal", -1, -2, opts={"split_segment": int(segc)})
    _check(oracle, "semiglobal", pairs, got, -1, -2)
    assert st["split"] == 1 and sp["tail_moves"] == 0 and sp["strips_taken"] > 0, sp


def test_split_matches_whole_walk(monkeypatch):
    """The same batch walked whole (BG_SPLIT=0, one workgroup per pair) and split: identical."""
    rng = random.Random(7)
    pairs = _pairs(rng, [(11000, 10000), (8000, 300), (5000, 9000)], rate=0.3)
    split, st1, _ = _run(pairs, "semiglobal", -1, -2, executes=3)
    whole, st0, _ = _run(pairs, "semiglobal", -1, -2, opts={"split": 0})
    assert st1["split"] == 1 and st0["split"] == 0
    assert split == whole


def test_split_exit_overflow_falls_back(oracle):
    """Scores too large for the exit pass's 13-bit value field (S - 2a = 32, near-identical
    pairs): the pass flags the pair and the tail walks it whole; still the reference's answer."""
    from biogarden_amd.alignment import score as score_mod
    from biogarden_amd import _native

    def big(x, y):
        return 30 if x == y else -5
    rng = random.Random(3)
    pairs = _pairs(rng, [(8000, 8000), (5000, 4000)], rate=0.02)
    sc, _ = score_mod.tabulate(big, pairs)
    got, st, sp = _run(pairs, "semiglobal", -1, -1, scoring=sc)
    _check(oracle, "semiglobal", pairs, got, -1, -1, scoring=oracle.scoring(big))
    assert st["split"] == 1 and st["tagged"] == 1, st
    assert sp["pairs_overflow"] >= 1, sp


def test_split_global_column0_paths(oracle):
    """Global pairs whose paths run up column 0 (seq2 much shorter than seq1): the chain carries
    exit 0 through the strips above, whose walks are pure up moves along the border."""
    rng = random.Random(11)
    pairs = [(rand_seq(rng, 9000, DNA), rand_seq(rng, 40, DNA)),
             (rand_seq(rng, 7000, DNA), rand_seq(rng, 3, DNA))]
    got, st, sp = _run(pairs, "global", -1, -2)
    _check(oracle, "global", pairs, got, -1, -2)
    assert st["split"] == 1 and sp["tail_moves"] == 0, sp


def test_split_exit_pass_beside_dp(oracle, monkeypatch):
    """The exit pass beside the DP (persistent workers on the CUs the WIDE DP leaves idle, inputs
    from the DP's epoch-tagged granules) against the pass after the DP: identical results, and
    the concurrent pass did the items (so the granule hand-off, not the fallback, is tested)."""
    rng = random.Random(23)
    pairs = _pairs(rng, [(20000, 19000), (9000, 9500)], rate=0.2)
    dg = {}
    conc, st, sp = _run(pairs, "semiglobal", -1, -2, executes=3, diag=dg, opts={"split_concurrent": 1})
    print("conc diag", dg, "split", sp, flush=True)
    _check(oracle, "semiglobal", pairs, conc, -1, -2)
    assert st["split"] == 1 and sp["tail_moves"] == 0 and sp["pairs_overflow"] == 0, sp
    assert dg["abandoned"] == 0 and dg["not_resident"] == 0, dg
    assert sp["items_beside_dp"] > 0, sp
    post, _, sp0 = _run(pairs, "semiglobal", -1, -2, opts={"split_concurrent": 0})
    assert sp0["items_beside_dp"] == 0 and sp0["tail_moves"] == 0, sp0
    assert post == conc


@pytest.mark.parametrize("depth,conc", [(1, None), (2, None), (3, None), (4, None), (3, "1"), (3, "0")])
def test_split_pipelined_two_dp_streams(oracle, monkeypatch, depth, conc):
    """WIDE batches executed back to back: consecutive DPs alternate two HIP streams and run side
    by side (the default at depth >= 2), with the exit pass beside the DP automatic (only when no
    other DP is in flight), forced on, or off; every pipeline depth returns the reference's answer
    for the last execute."""
    from biogarden_amd import _native
    rng = random.Random(100 + depth)
    pairs = _pairs(rng, [(15000, 14000), (6000, 300)], rate=0.2)
    h = _native.Handle(0)
    try:
        if conc is not None:
            h.set_option("split_concurrent", int(conc))
        h.set_pipeline(depth)
        h.prepare("semiglobal", pairs, _native.builtin_scoring(_native.BG_BLOSUM62), -1, -2)
        for _ in range(5):
            h.execute()
        got = h.fetch()
        sp = h.split_stats()
    finally:
        h.close()
    _check(oracle, "semiglobal", pairs, got, -1, -2)
    assert sp["tail_moves"] == 0, sp


def test_split_arena_reused_across_layouts(oracle):
    """One handle prepares a large split batch, then a smaller one with another layout (other
    lengths, strips and segments): the split arena is zeroed at every prepare, so no column
    number of the first batch can stand where the second one's epoch tags live — the strip walks
    still cover the whole traceback (a stale int equal to the epoch skipped items)."""
    from biogarden_amd import _native
    rng = random.Random(4242)
    big = _pairs(rng, [(16000, 15000), (9000, 12000)])
    small = _pairs(rng, [(7000, 5000), (5200, 3100), (3000, 6000)])
    sc = _native.builtin_scoring(_native.BG_BLOSUM62)
    h = _native.Handle(0)
    try:
        for pairs, reps in ((big, 2), (small, 3), (big[:1], 1)):
            h.prepare("semiglobal", pairs, sc, -1, -2)
            for _ in range(reps):
                h.execute()
            got = h.fetch()
            _check(oracle, "semiglobal", pairs, got, -1, -2)
            assert h.stats()["split"] == 1
            sp = h.split_stats()
            assert sp["pairs_overflow"] == 0 and sp["tail_moves"] == 0, sp
    finally:
        h.close()
