"""Substitution scores — mirrors src/alignment/score.rs of the reference.

`blosum62`, `pam250`, `unit` are callables S(a, b) on bytes (like the Rust fns taking &u8),
backed by the same 26x26 tables the HIP library carries (decoded from it through
bg_scoring_builtin, so the Python and device tables cannot drift apart).  Indices are
(byte - 65); bytes outside 'A'..'Z' raise IndexError where the reference panics (score.rs:40).
"""
from .. import _native


class ScoreTable:
    def __init__(self, name, which):
        self.__name__ = name
        self.which = which
        self._rows = None

    def _load(self):
        if self._rows is None:
            sc = _native.builtin_scoring(self.which)
            self._rows = [[sc.table[r * 32 + c] for c in range(26)] for r in range(26)]
        return self._rows

    def table(self):
        return [row[:] for row in self._load()]

    def __call__(self, a, b):
        a = a if isinstance(a, int) else ord(a)
        b = b if isinstance(b, int) else ord(b)
        if not (65 <= a <= 90 and 65 <= b <= 90):
            raise IndexError("score table index out of range (the reference panics)")
        return self._load()[a - 65][b - 65]

    def scoring(self):
        return _native.builtin_scoring(self.which)

    def __repr__(self):
        return "<score %s>" % self.__name__


blosum62 = ScoreTable("blosum62", _native.BG_BLOSUM62)
pam250 = ScoreTable("pam250", _native.BG_PAM250)
unit = ScoreTable("unit", _native.BG_UNIT)


def tabulate(score, seq1, seq2):
    """A.8: turn an arbitrary closure S(byte1, byte2) into bg_scoring by calling it once per
    distinct (byte of seq1, byte of seq2) pair.  A pair on which the closure raises is marked
    unscorable (the reference would panic the first time the DP reached it)."""
    if isinstance(score, ScoreTable):
        return score.scoring()
    syms = sorted(set(bytes(seq1)) | set(bytes(seq2)))
    if len(syms) > 32:
        raise ValueError("more than 32 distinct symbols")
    sc = _native.BgScoring()
    sc.alphabet_size = len(syms)
    for x in range(256):
        sc.code[x] = 0xFF
    bad = set()
    for i, x in enumerate(syms):
        sc.code[x] = i
    for i, x in enumerate(syms):
        for j, y in enumerate(syms):
            try:
                sc.table[i * 32 + j] = int(score(x, y))
            except Exception:
                bad.add(x)
                bad.add(y)
    for x in bad:
        sc.code[x] = 0xFF
    return sc
