"""Tile — mirrors src/ds/tile.rs:9-177: an ordered container of Sequences (FASTA sink and
batch input)."""
from .sequence import Sequence


class Tile:
    __slots__ = ("data",)

    def __init__(self, data=None):
        self.data = [s if isinstance(s, Sequence) else Sequence(s) for s in (data or [])]

    @classmethod
    def new(cls):
        return cls()

    def push(self, value):
        self.data.append(value)

    def pop(self):
        return self.data.pop() if self.data else None

    def remove(self, index):
        return self.data.pop(index)

    def size(self):
        return (len(self.data), len(self.data[0]))

    def len(self):
        return len(self.data)

    def is_empty(self):
        return not self.data

    def extend(self, other):
        self.data.extend(other.data)

    def __len__(self):
        return len(self.data)

    def __getitem__(self, i):
        return self.data[i]

    def __iter__(self):
        return iter(self.data)
