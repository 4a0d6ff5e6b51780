"""Sequence — mirrors src/ds/sequence.rs:10-257 of the reference.

`chain` is raw bytes (no case folding or validation); equality and hashing ignore `id`
(sequence.rs:104-117); Display prints the chain as UTF-8 (:251-257).
"""


class Sequence:
    __slots__ = ("chain", "id")

    def __init__(self, chain=b"", id=None):
        if isinstance(chain, Sequence):
            chain = chain.chain
        elif isinstance(chain, str):
            chain = chain.encode()
        self.chain = bytearray(chain)
        self.id = id

    # ---- constructors (sequence.rs:142-191)
    @classmethod
    def new(cls):
        return cls()

    @classmethod
    def from_record(cls, record):
        return cls(record.seq(), record.id())

    # ---- Vec-like surface (sequence.rs:17-47)
    def push(self, x):
        self.chain.append(x)

    def pop(self):
        return self.chain.pop() if self.chain else None

    def extend(self, other):
        self.chain.extend(other.chain if isinstance(other, Sequence) else other)

    def back(self):
        return self.chain[-1] if self.chain else None

    def len(self):
        return len(self.chain)

    def is_empty(self):
        return not self.chain

    def reverse(self):
        self.chain.reverse()

    def starts_with(self, prefix):
        return bytes(self.chain).startswith(bytes(prefix.chain))

    def to_bytes(self):
        return bytes(self.chain)

    # ---- traits
    def __len__(self):
        return len(self.chain)

    def __getitem__(self, i):
        return self.chain[i]

    def __iter__(self):
        return iter(self.chain)

    def __eq__(self, other):
        if isinstance(other, Sequence):
            return self.chain == other.chain
        if isinstance(other, (bytes, bytearray)):
            return bytes(self.chain) == bytes(other)
        if isinstance(other, str):
            return bytes(self.chain) == other.encode()
        return NotImplemented

    def __hash__(self):
        return hash(bytes(self.chain))

    def __str__(self):
        return self.chain.decode()

    def __repr__(self):
        return "Sequence(%r)" % bytes(self.chain)
