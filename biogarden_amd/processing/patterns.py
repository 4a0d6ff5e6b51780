"""processing::patterns::{longest_common_subsequence, shortest_common_supersequence}
(src/processing/patterns.rs:82-118, 198-235) on the MI355X.

The LCS match table is the global DP with byte equality scored +1 / -1 and open = extend = 0;
the reference's walk (a match always goes diagonal, otherwise up only when strictly greater than
left) is the traceback of that DP under the LCS tie rule, which the GPU's recomputing traceback
applies (bg_lcs_batch).  The subsequence is the seq1 residues of the diagonal columns.  The
supersequence interleaves both sequences around it exactly as the reference does (host-side,
O(n1 + n2)).  No CPU DP path; raises NativeUnavailable without the library or a GPU.
"""
from .. import _device
from ..ds.sequence import Sequence


def _bytes(s):
    return bytes(s.chain) if isinstance(s, Sequence) else bytes(s)


def longest_common_subsequence(seq1, seq2):
    """The reference's LCS of seq1 and seq2 as a Sequence (id None)."""
    return Sequence(_device.handle().lcs_batch([(_bytes(seq1), _bytes(seq2))])[0])


def longest_common_subsequence_batch(pairs):
    return [Sequence(x) for x in _device.handle().lcs_batch([(_bytes(a), _bytes(b)) for a, b in pairs])]


def _merge(s1, s2, lcs):
    # patterns.rs:199-235: before each LCS residue, the residues of seq1 then seq2 that differ
    # from it (the first equal one is consumed), then the residue; then both tails
    out = bytearray()
    i = j = 0
    for c in lcs:
        while i < len(s1):
            x = s1[i]
            i += 1
            if x == c:
                break
            out.append(x)
        while j < len(s2):
            x = s2[j]
            j += 1
            if x == c:
                break
            out.append(x)
        out.append(c)
    out += s1[i:]
    out += s2[j:]
    return bytes(out)


def shortest_common_supersequence(seq1, seq2):
    """The reference's shortest common supersequence as a Sequence (id None)."""
    s1, s2 = _bytes(seq1), _bytes(seq2)
    lcs = _device.handle().lcs_batch([(s1, s2)])[0]
    return Sequence(_merge(s1, s2, lcs))


def shortest_common_supersequence_batch(pairs):
    ps = [(_bytes(a), _bytes(b)) for a, b in pairs]
    return [Sequence(_merge(a, b, l)) for (a, b), l in zip(ps, _device.handle().lcs_batch(ps))]
