"""Streaming FASTA ingest (libbiogarden_gpu.so bg_fasta_*, biogarden_amd.io.fasta.BatchReader)
against the Python mirror of the reference reader (fasta.rs:95-135): same records (id, desc,
residues) on the reference fixtures and on generated files with the edge cases the reference's
rules cover — CRLF and trailing whitespace (trim_end), Unicode whitespace in headers, empty
lines, header-only records, the empty record that stops read_all, a first line without '>'
(the error) — at several block sizes so lines straddle block boundaries.  Host code only."""
import glob
import os
import random

import pytest

from conftest import REF_FIX


def _py_records(path):
    from biogarden_amd.io import fasta
    r = fasta.Reader.from_file(path)
    try:
        return [(x.id(), x.desc(), x.seq()) for x in r.records()]
    finally:
        r.close()


def _native_records(path, max_records, max_residues, block=None):
    from biogarden_amd.io import fasta
    old = os.environ.get("BG_FASTA_BLOCK")
    if block:
        os.environ["BG_FASTA_BLOCK"] = str(block)
    try:
        rd = fasta.BatchReader(path, max_records=max_records, max_residues=max_residues)
    finally:
        if block:
            if old is None:
                os.environ.pop("BG_FASTA_BLOCK")
            else:
                os.environ["BG_FASTA_BLOCK"] = old
    out, sizes = [], []
    try:
        for b in rd:
            sizes.append(len(b))
            out += [(x.id(), x.desc(), x.seq()) for x in b.records()]
    finally:
        rd.close()
    return out, sizes


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(REF_FIX, "input", "*.fasta"))))
def test_reference_fixtures(path):
    want = _py_records(path)
    got, _ = _native_records(path, 1, 1 << 30)
    assert got == want and len(want) >= 2


def _gen(rng, n):
    ws_tail = ["", " ", "\t", "\r", " \r", " ", "　 ", "\x0b"]
    lines = []
    for k in range(n):
        ident = "".join(rng.choice("ABCxyz0123_.|") for _ in range(rng.randint(0, 12)))
        head = ">" + (" " if rng.random() < 0.05 else "") + ident
        r = rng.random()
        if r < 0.3:
            head += rng.choice([" ", "\t", " "]) + "desc %d  x" % k
        elif r < 0.35:
            head += "  "
        lines.append(head + rng.choice(ws_tail))
        for _ in range(rng.choice([0, 1, 1, 2, 5, 30])):
            seq = "".join(rng.choice("ACGTNacgt") for _ in range(rng.choice([0, 1, 60, 61, 200])))
            lines.append(seq + rng.choice(ws_tail))
    eol = rng.choice(["\n", "\r\n"])
    return eol.join(lines) + (eol if rng.random() < 0.7 else "")


@pytest.mark.parametrize("seed", range(12))
def test_generated_files_all_block_sizes(tmp_path, seed):
    rng = random.Random(seed)
    text = _gen(rng, rng.randint(1, 60))
    path = tmp_path / "g.fa"
    path.write_bytes(text.encode("utf-8"))
    want = _py_records(str(path))
    for block in (1, 7, 64, 4096, None):
        for maxr, maxres in ((1, 1 << 30), (3, 1 << 30), (1 << 20, 100), (1 << 20, 1 << 30)):
            got, sizes = _native_records(str(path), maxr, maxres, block)
            assert got == want, (seed, block, maxr, maxres)
            assert all(s <= maxr for s in sizes)


def test_empty_record_stops_like_read_all(tmp_path):
    path = tmp_path / "e.fa"
    path.write_bytes(b">a\nAC\n>\n>b\nGG\n")
    assert _py_records(str(path)) == [("a", None, b"AC")]
    assert _native_records(str(path), 10, 100)[0] == [("a", None, b"AC")]


def test_first_line_without_header_is_an_error(tmp_path):
    path = tmp_path / "bad.fa"
    path.write_bytes(b"ACGT\n>a\nAC\n")
    with pytest.raises(IOError, match="Expected > at record start."):
        _py_records(str(path))
    with pytest.raises(IOError, match="Expected > at record start."):
        _native_records(str(path), 10, 100)


def test_missing_file(tmp_path):
    from biogarden_amd.io import fasta
    with pytest.raises(IOError):
        fasta.BatchReader(str(tmp_path / "nope.fa"))


def test_empty_file(tmp_path):
    path = tmp_path / "z.fa"
    path.write_bytes(b"")
    assert _native_records(str(path), 10, 100) == ([], [])


@pytest.mark.parametrize("data", [
    b">a\nAC\xffGT\n>b\nGG\n",              # a byte that never starts UTF-8
    b">a\xc3\n",                            # truncated two-byte form
    b">a\nACGT\n>b \xed\xa0\x80\nGG\n",     # a surrogate (U+D800) in the next header
    b">a\nAC\xc0\xafG\n",                   # overlong '/'
    b">a\nAC\xf4\x90\x80\x80\n",            # above U+10FFFF
])
def test_invalid_utf8_is_an_error(tmp_path, data):
    """BufRead::read_line fails on a line that is not UTF-8 (fasta.rs:97, 115): read_all returns
    Err(InvalidData).  Both readers raise, at every block size."""
    from biogarden_amd.io import fasta
    path = tmp_path / "u.fa"
    path.write_bytes(data)
    with pytest.raises(IOError, match=fasta.UTF8_ERROR):
        _py_records(str(path))
    for block in (1, 3, None):
        with pytest.raises(IOError, match=fasta.UTF8_ERROR):
            _native_records(str(path), 10, 100, block)


def test_valid_multibyte_utf8_is_accepted(tmp_path):
    path = tmp_path / "m.fa"
    path.write_bytes(">α β　desc\nAC\n>\U0001F600\nGT \n".encode("utf-8"))
    want = _py_records(str(path))
    assert want == [("α", "β　desc", b"AC"), ("\U0001F600", None, b"GT")]
    assert _native_records(str(path), 10, 100, 2)[0] == want


@pytest.mark.parametrize("maxr,maxres", [(0, 100), (10, 0)])
def test_zero_batch_limits_are_refused(tmp_path, maxr, maxres):
    from biogarden_amd.io import fasta
    path = tmp_path / "z.fa"
    path.write_bytes(b">a\nAC\n")
    with pytest.raises(ValueError):
        fasta.BatchReader(str(path), max_records=maxr, max_residues=maxres)


def test_zero_max_residues_is_refused_by_the_abi(tmp_path):
    import ctypes
    from biogarden_amd import _native
    path = tmp_path / "z.fa"
    path.write_bytes(b">a\nAC\n")
    L = _native.lib()
    err = ctypes.c_int(0)
    r = L.bg_fasta_open(str(path).encode(), ctypes.byref(err))
    try:
        b = _native.BgFastaBatch()
        assert L.bg_fasta_next_batch(r, 10, 0, ctypes.byref(b)) == -1
        assert L.bg_fasta_next_batch(r, 10, 100, ctypes.byref(b)) == 1
    finally:
        L.bg_fasta_close(r)
