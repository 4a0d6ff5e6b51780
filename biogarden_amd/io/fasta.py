"""FASTA reader/writer — mirrors src/io/fasta.rs:21-320 of the reference.

Reader.read (fasta.rs:95-123): a record starts at a line beginning with '>' (else IOError
"Expected > at record start."); id = first whitespace-delimited token of the header, desc =
the rest; the sequence is the concatenation of the following lines with trailing whitespace
removed (`trim_end`), up to EOF or the next '>'.  At EOF the record comes back empty.
"""
from ..ds.sequence import Sequence


class Record:
    __slots__ = ("_id", "_desc", "_seq")

    def __init__(self, id="", desc=None, seq=b""):
        self._id = id
        self._desc = desc
        self._seq = bytearray(seq.encode() if isinstance(seq, str) else seq)

    @classmethod
    def new(cls):
        return cls()

    @classmethod
    def with_attrs(cls, id, desc, seq):
        return cls(id, desc, seq)

    def is_empty(self):
        return not self._id and self._desc is None and not self._seq

    def check(self):
        if not self._id:
            raise ValueError("Expecting id for Fasta record.")
        if any(c > 127 for c in self._seq):
            raise ValueError("Non-ascii character found in sequence.")

    def id(self):
        return self._id

    def desc(self):
        return self._desc

    def seq(self):
        return bytes(self._seq)

    def clear(self):
        self._id = ""
        self._desc = None
        self._seq = bytearray()

    def __str__(self):
        header = self._id if self._desc is None else "%s %s" % (self._id, self._desc)
        return ">%s\n%s\n" % (header, self._seq.decode())


# char::is_whitespace (Unicode White_Space), which str::trim_end and the header's
# splitn(2, char::is_whitespace) use (fasta.rs:110, :119); Python's str.isspace differs
# (it also takes U+001C-001F)
_WS = frozenset("\t\n\x0b\x0c\r \x85\xa0\u1680\u2000\u2001\u2002\u2003\u2004\u2005"
                "\u2006\u2007\u2008\u2009\u200a\u2028\u2029\u202f\u205f\u3000")


# std's message for BufRead::read_line on bytes that are not UTF-8 (io::ErrorKind::InvalidData)
UTF8_ERROR = "stream did not contain valid UTF-8"


def _trim_end(s):
    return s.rstrip("".join(_WS))


class Reader:
    def __init__(self, stream):
        self._r = stream
        self._line = ""

    @classmethod
    def from_file(cls, path):
        try:
            return cls(open(path, "r", newline="", encoding="utf-8"))
        except OSError as e:
            raise IOError("Failed to read fasta from %r" % (str(path),)) from e

    def _readline(self):
        try:
            return self._r.readline()
        except UnicodeDecodeError as e:
            raise IOError(UTF8_ERROR) from e

    def read(self, record):
        record.clear()
        if not self._line:
            self._line = self._readline()
            if not self._line:
                return
        if not self._line.startswith(">"):
            raise IOError("Expected > at record start.")
        head = _trim_end(self._line[1:])
        # splitn(2, char::is_whitespace): id is the text before the FIRST whitespace char
        cut = next((i for i, ch in enumerate(head) if ch in _WS), None)
        if cut is None:
            record._id, record._desc = head, None
        else:
            record._id, record._desc = head[:cut], head[cut + 1:]
        while True:
            self._line = self._readline()
            if not self._line or self._line.startswith(">"):
                break
            record._seq.extend(_trim_end(self._line).encode())

    def read_all(self, tile):
        record = Record()
        while True:
            self.read(record)
            if record.is_empty():
                break
            tile.push(Sequence(record.seq(), record.id()))

    def records(self):
        while True:
            rec = Record()
            self.read(rec)
            if rec.is_empty():
                return
            yield rec

    def close(self):
        self._r.close()


class Writer:
    def __init__(self, stream):
        self._w = stream

    @classmethod
    def to_file(cls, path):
        return cls(open(path, "w", newline=""))

    def write_record(self, record):
        self.write(record.id(), record.desc(), record.seq())

    def write(self, id, desc, seq):
        self._w.write(">" + id)
        if desc is not None:
            self._w.write(" " + desc)
        self._w.write("\n")
        self._w.write(bytes(seq).decode())
        self._w.write("\n")

    def flush(self):
        self._w.flush()

    def close(self):
        self._w.close()


class FastaBatch:
    """One batch of records from BatchReader: residues back to back in `seq` (bytes), record r
    at seq[offsets[r]:offsets[r+1]]; ids / descriptions as the reference's Record has them."""
    __slots__ = ("seq", "offsets", "ids", "descs")

    def __init__(self, seq, offsets, ids, descs):
        self.seq = seq
        self.offsets = offsets
        self.ids = ids
        self.descs = descs

    def __len__(self):
        return len(self.ids)

    def sequence(self, r):
        return self.seq[self.offsets[r]:self.offsets[r + 1]]

    def records(self):
        return [Record(self.ids[r], self.descs[r], self.sequence(r)) for r in range(len(self))]

    def tile(self):
        from ..ds.tile import Tile
        t = Tile()
        for r in range(len(self)):
            t.push(Sequence(self.sequence(r), self.ids[r]))
        return t


class BatchReader:
    """Streaming FASTA ingest for the batch aligner (native, libbiogarden_gpu.so bg_fasta_*):
    the file is read in large blocks and returned as FastaBatch objects of at most
    `max_records` records / about `max_residues` residues, with read_all's record rules
    (fasta.rs:95-135).  Feed a batch to AlignStream / Handle.prepare_packed without per-record
    copies."""

    def __init__(self, path, max_records=65536, max_residues=64 << 20):
        import ctypes
        from .. import _native
        if max_records < 1 or max_residues < 1:
            raise ValueError("max_records and max_residues must be positive")
        self._n = _native
        err = ctypes.c_int(0)
        self._r = _native.lib().bg_fasta_open(str(path).encode(), ctypes.byref(err))
        if not self._r:
            raise IOError("Failed to read fasta from %r" % (str(path),))
        self.max_records = max_records
        self.max_residues = max_residues

    def next_batch(self):
        import ctypes
        import numpy as np
        b = self._n.BgFastaBatch()
        rc = self._n.lib().bg_fasta_next_batch(self._r, self.max_records, self.max_residues,
                                               ctypes.byref(b))
        if rc < 0:
            if rc == -8:
                raise IOError("Expected > at record start.")
            if rc == -9:
                raise IOError(UTF8_ERROR)
            self._n.check(rc)
        n = b.n
        if n == 0:
            return None
        offs = np.ctypeslib.as_array(b.seq_off, shape=(n + 1,)).copy()
        seq = ctypes.string_at(b.seq, int(offs[-1])) if offs[-1] else b""
        ido = np.ctypeslib.as_array(b.id_off, shape=(n,))
        dso = np.ctypeslib.as_array(b.desc_off, shape=(n,))
        ids, descs = [], []
        for r in range(n):
            ids.append(ctypes.string_at(b.text + int(ido[r])).decode("utf-8", "surrogateescape"))
            d = int(dso[r])
            descs.append(None if d == 0xFFFFFFFFFFFFFFFF else
                         ctypes.string_at(b.text + d).decode("utf-8", "surrogateescape"))
        return FastaBatch(seq, offs, ids, descs)

    def __iter__(self):
        while True:
            batch = self.next_batch()
            if batch is None:
                return
            yield batch

    def close(self):
        if self._r:
            self._n.lib().bg_fasta_close(self._r)
            self._r = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def read_tile(path):
    """Reads every record of a FASTA file into a Tile (the reference's read_all)."""
    from ..ds.tile import Tile
    t = Tile()
    r = Reader.from_file(path)
    try:
        r.read_all(t)
    finally:
        r.close()
    return t
