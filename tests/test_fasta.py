"""io::fasta reader/writer restatement (fasta.rs:95-201) against the fixtures and edge cases."""
import io
import os

import pytest

from conftest import REF_FIX, read_fasta


def test_reader_matches_fixtures():
    from biogarden_amd.io import fasta
    for mode in ("global", "local", "fitting", "overlap", "semiglobal"):
        for d in ("input", "output"):
            p = os.path.join(REF_FIX, d, "%s_alignment.fasta" % mode)
            t = fasta.read_tile(p)
            ref = read_fasta(p)
            assert [s.id for s in t] == [r[0] for r in ref]
            assert [bytes(s.chain) for s in t] == [r[1] for r in ref]


def test_reader_semantics():
    from biogarden_amd.io import fasta
    r = fasta.Reader(io.StringIO(">id1 some desc  \nACGT  \r\nGG\n>id2\n\nTT\n"))
    rec = fasta.Record()
    r.read(rec)
    assert (rec.id(), rec.desc(), rec.seq()) == ("id1", "some desc", b"ACGTGG")
    r.read(rec)
    assert (rec.id(), rec.desc(), rec.seq()) == ("id2", None, b"TT")
    r.read(rec)
    assert rec.is_empty()
    with pytest.raises(IOError):
        fasta.Reader(io.StringIO("ACGT\n")).read(fasta.Record())


def test_writer_roundtrip():
    from biogarden_amd.io import fasta
    buf = io.StringIO()
    w = fasta.Writer(buf)
    w.write("x", "d e", b"ACGT")
    w.write("y", None, b"")
    r = fasta.Reader(io.StringIO(buf.getvalue()))
    recs = list(r.records())
    assert [(x.id(), x.desc(), x.seq()) for x in recs] == [("x", "d e", b"ACGT"), ("y", None, b"")]


def test_sequence_and_tile():
    from biogarden_amd.ds import Sequence, Tile
    s = Sequence("ACGT", id="a")
    assert s == Sequence(b"ACGT", id="b")          # equality ignores id (sequence.rs:113-117)
    assert hash(s) == hash(Sequence("ACGT"))
    s.push(ord("A"))
    s.reverse()
    assert str(s) == "ATGCA"
    t = Tile([Sequence("AC"), Sequence("G")])
    assert len(t) == 2 and t.size() == (2, 2) and t[1] == "G"


def test_tabulate_closure_panics_per_pair():
    """A.8: a closure is evaluated on set(seq1) x set(seq2) only; the pairs it panics on make
    exactly the pairs whose DP would reach them unscorable."""
    from biogarden_amd.alignment import score

    def s(x, y):
        if (x, y) == (ord("A"), ord("T")):
            raise IndexError("panic")
        return 2 if x == y else -1

    sc, panics = score.tabulate(s, [(b"AC", b"GT"), (b"TT", b"AA")])
    assert panics == {(ord("A"), ord("T"))}
    assert sc.alphabet_size == 4
    assert score.pair_panics(panics, b"AC", b"GT")
    assert not score.pair_panics(panics, b"TT", b"AA")
    assert not score.pair_panics(panics, b"", b"T")
    assert sc.table[sc.code[ord("C")] * 32 + sc.code[ord("T")]] == -1
    tab, none = score.tabulate(score.blosum62, [(b"AC", b"GT")])
    assert none == set() and tab.alphabet_size == 26
