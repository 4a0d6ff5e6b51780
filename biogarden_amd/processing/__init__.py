"""processing — the reference's src/processing module, restricted to the alignment-DP patterns
(longest_common_subsequence, shortest_common_supersequence)."""
from . import patterns  # noqa: F401
