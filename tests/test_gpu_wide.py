"""GPU parity of the WIDE strip pipeline (a few long pairs spread over many workgroups,
bg_dp_tag_kernel<R, true, true> with the conveyor step) at the edges C3's shape
does not reach: every linear-gap mode, strip heights 2..10, seq2 lengths around the 64-column
block (1, 5, 63, 64, 65, 127, 128, 129) and long, and small pairs riding in the same batch.
Score and both strings against oracle.align(..., exact=True)."""
import random

import pytest

from parity_util import DNA, check_batch, mutate, rand_seq

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def aligner():
    from biogarden_amd.alignment.aligner import SequenceAligner
    al = SequenceAligner(0)
    yield al
    al.close()


@pytest.mark.parametrize("R", [2, 3, 4, 5, 8, 10])
@pytest.mark.parametrize("mode,a,b", [("semiglobal", -1, -2), ("global", -1, -2), ("fitting", -2, -2),
                                      ("overlap", -1, -3)])
def test_wide_edges(aligner, oracle, R, mode, a, b):
    rng = random.Random(R * 131 + len(mode) + a)
    pairs = []
    for n1, n2 in ((4100, 1), (4100, 5), (4160, 63), (4200, 64), (4300, 65), (5000, 127),
                   (4097, 128), (4500, 129), (5200, 1900), (1, 700), (300, 280), (4096, 4096)):
        s1 = rand_seq(rng, n1, DNA)
        s2 = (mutate(rng, s1, DNA, 0.15) * 2)[:n2] if n2 > 5 else rand_seq(rng, n2, DNA)
        pairs.append((s1, s2))
    aligner.set_tuning(R, 0)          # strip height only: the WIDE planner still places the pairs
    try:
        check_batch(aligner, oracle, mode, pairs, "blosum62", a, b, fresh=False)
        st = aligner.stats()
        assert st["wide"] == 1 and st["checkpoint"] == 1 and st["R"] == R, st
    finally:
        aligner.set_tuning(0, 0)


@pytest.mark.parametrize("depth", [2, 3])
def test_wide_repeated_executes_alternating_traceback_streams(oracle, depth):
    """A WIDE batch executed back to back: its tracebacks alternate between two HIP streams and
    overlap each other (bg_batch_execute), each reading its own arena slot; the fetched result of
    the last execute must still be the reference's, for every pipeline depth."""
    from biogarden_amd import _native
    rng = random.Random(depth)
    pairs = []
    for n1, n2 in ((9000, 8800), (4200, 300), (6000, 6100)):
        s1 = rand_seq(rng, n1, DNA)
        pairs.append((s1, mutate(rng, s1, DNA, 0.2)[:n2]))
    h = _native.Handle(0)
    try:
        h.set_pipeline(depth)
        h.prepare("semiglobal", pairs, _native.builtin_scoring(_native.BG_BLOSUM62), -1, -2)
        assert h.stats()["wide"] == 1
        for _ in range(5):
            h.execute()
        got = h.fetch()
        for (s1, s2), r in zip(pairs, got):
            st, sc, o1, o2 = oracle.align("semiglobal", s1, s2, "blosum62", -1, -2, exact=True)
            assert st == 0 and r["status"] in (0, 4)
            assert (r["score"], r["aligned1"], r["aligned2"]) == (sc, o1, o2)
    finally:
        h.close()
