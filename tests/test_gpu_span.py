"""SPAN (bg_dp_tag_kernel<R, 2, true>, round 6): batches with fewer pairs than CUs (one batch of
M strong-scaled over 2-8 GPUs leaves 128-32 pairs per GPU) spread each pair's strips over a
group of many-wave workgroups, handing the boundary row to the next workgroup through HBM at
every W-th strip.  Results must not change: score and both strings against the oracle, and
identical to the plan without it (bg_set_option span = 0: WIDE lone-wave groups or one workgroup
per pair), at every strip height, in
the four linear-path modes, with pairs of unequal sizes (groups in proportion to cells), strips
that wrap to a second round, and empty pairs beside them."""
import random

import pytest

from parity_util import DNA, check_results, mutate, rand_seq, sample_indices

pytestmark = pytest.mark.gpu


def _run(mode, pairs, a, b, span, R=0, executes=1, split=None):
    from biogarden_amd import _native
    h = _native.Handle(0)
    try:
        h.set_option("span", span)
        h.set_option("split", split)
        if R:
            h.set_tuning(R, 0)
        h.prepare(mode, pairs, _native.builtin_scoring(_native.BG_BLOSUM62), a, b)
        for _ in range(executes):
            h.execute()
        return h.fetch(), h.stats()
    finally:
        h.close()


def _key(r):
    return (r["status"], r["score"], r["aligned1"], r["aligned2"])


def _pairs(seed, shapes, rate=0.12):
    rng = random.Random(seed)
    out = []
    for n1, n2 in shapes:
        s1 = rand_seq(rng, n1, DNA)
        s2 = (mutate(rng, s1, DNA, rate) + rand_seq(rng, n2, DNA))[:n2] if n2 > 8 else rand_seq(rng, n2, DNA)
        out.append((s1, s2))
    return out


@pytest.mark.parametrize("R", [2, 3, 4, 5, 8, 10])
def test_span_matches_one_workgroup_and_oracle(oracle, R):
    shapes = [(6000, 5000), (5200, 6100), (3000, 7000), (7000, 900), (4100, 4100), (2500, 2600)] * 3
    pairs = _pairs(100 + R, shapes)
    got, st = _run("semiglobal", pairs, -1, -2, 1, R=R, executes=2, split=1 if R % 2 else None)
    # the split traceback on request, at every other R
    assert st["wide"] == 2 and st["R"] == R and st["workgroups"] > len(pairs), st
    assert st["split"] == (1 if R % 2 else 0), st
    ref, st0 = _run("semiglobal", pairs, -1, -2, 0, R=R)      # WIDE (lone waves) or one per pair
    assert st0["wide"] != 2, st0
    diff = [p for p in range(len(pairs)) if _key(got[p]) != _key(ref[p])]
    assert not diff, diff[:10]
    check_results(oracle, "semiglobal", pairs, [_as_res(r) for r in got], "blosum62", -1, -2,
                  sample=sample_indices(len(pairs), 4, R))


@pytest.mark.parametrize("mode,a,b", [("global", -2, -2), ("fitting", -1, -1), ("overlap", -1, -3),
                                      ("semiglobal", -3, -3)])
@pytest.mark.parametrize("split", [None, 1])
def test_span_modes_vs_oracle(oracle, mode, a, b, split):
    shapes = [(4000, 3500), (3900, 3000), (2000, 1500), (5000, 400), (64, 5000), (0, 300), (300, 0)]
    if mode == "fitting":
        shapes = [(4000, 3500), (3900, 3000), (2000, 1500), (5000, 400), (4500, 64), (0, 0), (300, 0)]
    pairs = _pairs(7 + len(mode) + a, shapes * 2)
    got, st = _run(mode, pairs, a, b, 1, R=2, split=split)
    assert st["wide"] == 2 and st["split"] == (1 if split == 1 else 0), st
    ref, _ = _run(mode, pairs, a, b, 0, R=2)
    assert [_key(r) for r in got] == [_key(r) for r in ref]
    check_results(oracle, mode, pairs, [_as_res(r) for r in got], "blosum62", a, b)


def test_span_planner_picks_groups_for_few_long_pairs():
    """The automatic plan: 64 pairs of 10 k x 10 k (M's share at 4 GPUs) spread over groups."""
    from tools import workloads as w
    pairs = w.metric_pairs(64, 10000, 10000, seed=w.SEED0 + 99)
    got, st = _run("semiglobal", pairs, -1, -2, -1)
    assert st["wide"] == 2 and st["workgroups"] >= 2 * len(pairs) and st["split"] == 0, st
    assert all(r["status"] == 0 for r in got)


def _as_res(r):
    """A fetch() dict in the shape check_results takes (the facade's (score, a1, a2) result)."""
    from biogarden_amd.alignment.aligner import AlignmentResult
    from biogarden_amd.ds.sequence import Sequence
    return AlignmentResult(r["score"], Sequence(r["aligned1"]), Sequence(r["aligned2"]),
                           status=r["status"], end=r["end"], start=r["start"])
