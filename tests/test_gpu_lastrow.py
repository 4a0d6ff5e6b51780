"""The last strip of the score-only DP repeats row n1 below it (bg_tag_kernel.hip, round 5): the
rows under row n1 get profile bytes -128 and row n1's column-0 value, so they copy row n1 and the
lane holding row n1 hands it down as its last row without a select per row and step.  Row n1
drives the end cell (the last row's maximum, aligner.rs:369-389) and the traceback never walks
below it, so results must not change: score and both strings against the oracle with row n1 in
every row of a lane and in lanes of every 16-lane group, at every strip height, in the four modes
that take the linear path (a >= b)."""
import random

import pytest

from parity_util import DNA, check_batch, mutate, rand_seq

pytestmark = pytest.mark.gpu


def _pairs(seed, lens, mode):
    rng = random.Random(seed)
    out = []
    for x, n1 in enumerate(lens):
        s1 = rand_seq(rng, n1, DNA)
        s2 = mutate(rng, s1, DNA, 0.15) if x % 3 else rand_seq(rng, max(1, n1 + rng.randint(-150, 150)), DNA)
        if mode == "fitting" and len(s2) > len(s1):
            s2 = s2[:len(s1)]
        out.append((s1, s2))
    return out


@pytest.mark.parametrize("R", [2, 3, 4, 5, 8, 10])
@pytest.mark.parametrize("mode,a,b", [("semiglobal", -1, -2), ("global", -2, -2), ("fitting", -1, -1),
                                      ("overlap", -1, -3)])
def test_last_strip_row_n1_everywhere(oracle, R, mode, a, b):
    from biogarden_amd.alignment.aligner import SequenceAligner
    S = 64 * R
    # row n1 at lane offsets 0, 15, 16, 31, 47, 63 and row offsets 0 .. R - 1 of the last strip
    lens = [S + 1 + lane * R + (lane % R) for lane in (0, 15, 16, 31, 47, 63)] + [S - 1, 2 * S, 2 * S + 5]
    pairs = _pairs(100 * R + len(mode), lens, mode)
    al = SequenceAligner(0)
    try:
        al.set_tuning(R, 2)
        res = check_batch(al, oracle, mode, pairs, "blosum62", a, b, sample=list(range(len(pairs))))
        st = al.stats()
        assert st["R"] == R and st["tagged"] == 1 and st["checkpoint"] == 1 and st["wide"] == 0, st
        assert all(r.status in (0, 4) for r in res)
    finally:
        al.close()
