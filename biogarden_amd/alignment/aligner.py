"""SequenceAligner — mirrors src/alignment/aligner.rs of the reference, on the MI355X.

Same method names, argument meaning and error behaviour as the Rust struct:

    aligner = SequenceAligner()                                   # aligner.rs:44 / Default :605
    score, s1, s2 = aligner.global_alignment(seq1, seq2, blosum62, -11, -1)        # :84
    aligner.local_alignment / fitting_alignment / overlap_alignment / semiglobal_alignment
                                                                  # :150, :216, :290, :351

Errors: InvalidArgumentRange / InvalidInputSize exactly where the reference returns them;
ReferencePanic where the reference panics or hangs.  Every call runs the HIP kernels of
libbiogarden_gpu.so; there is no CPU path.
"""
from .. import _native
from ..ds.sequence import Sequence
from ..error import InvalidArgumentRange, InvalidInputSize, ReferencePanic
from . import score as _score


class AlignmentResult(tuple):
    """(score, s1_aligned, s2_aligned) plus .status/.end/.start for batch callers."""

    def __new__(cls, score, a1, a2, status=0, end=(0, 0), start=(0, 0)):
        self = super().__new__(cls, (score, a1, a2))
        self.status = status
        self.end = end
        self.start = start
        return self


def _raise_for(status, res):
    if status == _native.BG_INVALID_ARGUMENT_RANGE:
        raise InvalidArgumentRange("The provided has is within an unsupported range!")
    if status == _native.BG_INVALID_INPUT_SIZE:
        raise InvalidInputSize("Provided inputs have invalid size!")
    if status == _native.BG_UNSCORABLE:
        raise ReferencePanic("score closure index out of range", None)
    if status == _native.BG_REF_DIVERGENT:
        raise ReferencePanic("the reference SequenceAligner panics or hangs on this input", res)
    if status == _native.BG_INTERNAL:
        raise RuntimeError("biogarden_gpu: traceback recomputation timed out (internal error)")


def _as_bytes(s):
    if isinstance(s, Sequence):
        return bytes(s.chain)
    if isinstance(s, str):
        return s.encode()
    return bytes(s)


class SequenceAligner:
    def __init__(self, device=None):
        if device is None:
            device = 0
        self._h = _native.Handle(device)

    @classmethod
    def new(cls, device=None):
        return cls(device)

    def set_tuning(self, R=0, waves=0):
        self._h.set_tuning(R, waves)

    def set_option(self, name, value):
        """bg_set_option (planner / traceback choices, never results): see _native.OPTIONS."""
        self._h.set_option(name, value)

    def options(self, **kw):
        return self._h.options(**kw)

    # ---------------------------------------------------------------- batch (Tile) form
    def align_batch(self, mode, pairs, score, a, b, strict=False):
        """Aligns many (seq1, seq2) pairs with one call.  Returns AlignmentResult per pair;
        with strict=True the first non-ok status raises like the single-pair methods."""
        pairs = [(_as_bytes(x), _as_bytes(y)) for x, y in pairs]
        sc, panics = _score.tabulate(score, pairs)
        out = self._h.align_batch(mode, pairs, sc, int(a), int(b))
        res = []
        for (s1, s2), r in zip(pairs, out):
            if r["status"] == 0 and _score.pair_panics(panics, s1, s2):
                r = dict(r, status=_native.BG_UNSCORABLE)
            ar = AlignmentResult(r["score"], Sequence(r["aligned1"]), Sequence(r["aligned2"]),
                                 r["status"], r["end"], r["start"])
            if strict and r["status"]:
                _raise_for(r["status"], ar)
            res.append(ar)
        return res

    def _one(self, mode, seq1, seq2, score, a, b):
        s1, s2 = _as_bytes(seq1), _as_bytes(seq2)
        sc, panics = _score.tabulate(score, [(s1, s2)])
        r = self._h.align_batch(mode, [(s1, s2)], sc, int(a), int(b))[0]
        if r["status"] == 0 and _score.pair_panics(panics, s1, s2):
            r = dict(r, status=_native.BG_UNSCORABLE)
        res = (r["score"], Sequence(r["aligned1"]), Sequence(r["aligned2"]))
        _raise_for(r["status"], res)
        return res

    # ---------------------------------------------------------------- reference surface
    def global_alignment(self, seq1, seq2, score, a, b):
        return self._one("global", seq1, seq2, score, a, b)

    def local_alignment(self, seq1, seq2, score, a, b):
        return self._one("local", seq1, seq2, score, a, b)

    def fitting_alignment(self, seq1, seq2, score, a, b):
        return self._one("fitting", seq1, seq2, score, a, b)

    def overlap_alignment(self, seq1, seq2, score, a, b):
        return self._one("overlap", seq1, seq2, score, a, b)

    def semiglobal_alignment(self, seq1, seq2, score, a, b):
        return self._one("semiglobal", seq1, seq2, score, a, b)

    def stats(self):
        return self._h.stats()

    @property
    def buffer_size(self):
        """(rows, cols) of the reference aligner's scratch after the calls so far (aligner.rs:30):
        (1024, 1024) when new, (len1+1, len2+1) after a call that did not fit (:92-94)."""
        return self._h.buffer_size()

    def close(self):
        self._h.close()
