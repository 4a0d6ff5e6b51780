"""analysis::seq::edit_distance (src/analysis/seq.rs:105-130) on the MI355X.

The unit-cost Levenshtein recurrence is the linear-gap global DP with byte equality scored
0 / -1 and open = extend = -1, so edit_distance = -score of that alignment.  It runs on the
aligner's GPU kernels (score only, no traceback) through bg_edit_distance_batch; there is no CPU
path.  Raises NativeUnavailable without the library or a GPU.
"""
from .. import _device
from ..ds.sequence import Sequence


def _bytes(s):
    return bytes(s.chain) if isinstance(s, Sequence) else bytes(s)


def edit_distance(seq1, seq2):
    """Ok(usize) of the reference: the minimum number of substitutions, insertions and
    deletions turning seq1 into seq2 (raw bytes, no case folding)."""
    return _device.handle().edit_distance_batch([(_bytes(seq1), _bytes(seq2))])[0]


def edit_distance_batch(pairs):
    """edit_distance over many pairs in one GPU batch."""
    return _device.handle().edit_distance_batch([(_bytes(a), _bytes(b)) for a, b in pairs])
