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


def tabulate(score, pairs):
    """A.8: turn an arbitrary closure S(byte1, byte2) into bg_scoring by calling it once per
    distinct (byte of a seq1, byte of a seq2) pair of the batch.  Returns (scoring, panics):
    `panics` is the set of (byte1, byte2) on which the closure raised; a pair whose
    set(seq1) x set(seq2) meets it is one where the reference panics (status 3, see
    pair_panics).  Built-in tables need no evaluation."""
    if isinstance(score, ScoreTable):
        return score.scoring(), set()
    xs = set()
    ys = set()
    for s1, s2 in pairs:
        xs.update(bytes(s1))
        ys.update(bytes(s2))
    syms = sorted(xs | ys)
    if len(syms) > 32:
        # beyond the 32 x 32 bg_scoring: a k x k table over every byte the batch uses
        k = len(syms)
        code = [0xFFFF] * 256
        for i, x in enumerate(syms):
            code[x] = i
        table = [0] * (k * k)
        panics = set()
        for x in sorted(xs):
            for y in sorted(ys):
                try:
                    table[code[x] * k + code[y]] = int(score(x, y))
                except Exception:
                    panics.add((x, y))
        return _native.WideScoring(code, k, table), panics
    sc = _native.BgScoring()
    sc.alphabet_size = len(syms)
    for x in range(256):
        sc.code[x] = 0xFF
    for i, x in enumerate(syms):
        sc.code[x] = i
    panics = set()
    for x in sorted(xs):
        for y in sorted(ys):
            try:
                sc.table[sc.code[x] * 32 + sc.code[y]] = int(score(x, y))
            except Exception:
                panics.add((x, y))
    return sc, panics


def pair_panics(panics, seq1, seq2):
    """True when the reference DP would evaluate a panicking (byte1, byte2) on this pair."""
    if not panics or not seq1 or not seq2:
        return False
    a, b = set(bytes(seq1)), set(bytes(seq2))
    return any(x in a and y in b for x, y in panics)
