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


def _trim_end(s):
    return s.rstrip()


class Reader:
    def __init__(self, stream):
        self._r = stream
        self._line = ""

    @classmethod
    def from_file(cls, path):
        try:
            return cls(open(path, "r", newline=""))
        except OSError as e:
            raise IOError("Failed to read fasta from %r" % (str(path),)) from e

    def read(self, record):
        record.clear()
        if not self._line:
            self._line = self._r.readline()
            if not self._line:
                return
        if not self._line.startswith(">"):
            raise IOError("Expected > at record start.")
        head = _trim_end(self._line[1:])
        # splitn(2, char::is_whitespace): id is the text before the FIRST whitespace char
        cut = next((i for i, ch in enumerate(head) if ch.isspace()), None)
        if cut is None:
            record._id, record._desc = head, None
        else:
            record._id, record._desc = head[:cut], head[cut + 1:]
        while True:
            self._line = self._r.readline()
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
