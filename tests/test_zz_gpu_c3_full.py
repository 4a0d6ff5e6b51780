"""C3 at full size, string for string (SURVEY §8(d) configs[2]: one 100 kbp x 100 kbp semiglobal
alignment, blosum62 -1/-2; reference semantics src/alignment/aligner.rs:351-435).

The GPU aligns workloads.c3_pair() through the product path (WIDE DP + split traceback); the
reference-faithful oracle (oracle/refcpu.c with the reference's six full matrices, one core,
~80 s) aligns the same pair, and score, end cell and both 124 k-column strings must be
identical.  The oracle needs ~150 GB of host memory (15 B/cell), so the test runs only where
MemAvailable >= 160 GiB (the MI355X boxes) and is skipped elsewhere.  The file name puts it
last in collection, so a failure here cannot hide the other GPU tests."""
import pytest

pytestmark = pytest.mark.gpu


def _mem_available_gib():
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemAvailable"):
                    return int(line.split()[1]) / 2 ** 20
    except OSError:
        pass
    return 0.0


@pytest.mark.timeout(900)
@pytest.mark.skipif(_mem_available_gib() < 160, reason="the reference's matrices need ~150 GB")
def test_C3_full_size_strings_equal_reference(oracle):
    from biogarden_amd.alignment import score
    from biogarden_amd.alignment.aligner import SequenceAligner
    from tools import workloads
    (s1, s2), = workloads.c3_pair()
    al = SequenceAligner(0)
    try:
        r, = al.align_batch("semiglobal", [(s1, s2)], score.blosum62, -1, -2)
        st = al.stats()
    finally:
        al.close()
    assert st["wide"] == 1 and st["tagged"] == 1, st
    ost, osc, o1, o2 = oracle.Aligner(exact=False).align("semiglobal", s1, s2, "blosum62", -1, -2)
    assert ost == 0 and r.status == 0, (ost, r.status)
    assert r[0] == osc
    assert bytes(r[1].chain) == o1 and bytes(r[2].chain) == o2
