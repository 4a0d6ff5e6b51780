"""GPU parity of the §8(f) widening rows that run on the alignment DP:
analysis::seq::edit_distance (src/analysis/seq.rs:105-130) and
processing::patterns::{longest_common_subsequence, shortest_common_supersequence}
(src/processing/patterns.rs:82-118, 198-235), through bg_edit_distance_batch / bg_lcs_batch.
Bit-exact against the oracle (oracle/refcpu.c), itself pinned by the reference's goldens
(tests/integration.rs:69-74, 135-149) and doctests.
"""
import os
import random

import pytest

from conftest import REF_FIX, read_fasta

pytestmark = pytest.mark.gpu

DNA = b"ACGT"
PROT = b"ACDEFGHIKLMNPQRSTVWY"


def rand_seq(rng, n, alpha):
    return bytes(rng.choice(alpha) for _ in range(n))


def mutate(rng, s, alpha, rate=0.2):
    out = bytearray()
    for ch in s:
        r = rng.random()
        if r < rate / 3:
            continue
        if r < 2 * rate / 3:
            out.append(rng.choice(alpha))
        out.append(rng.choice(alpha) if rng.random() < rate / 3 else ch)
    return bytes(out)


def test_reference_goldens():
    from biogarden_amd.analysis.seq import edit_distance
    from biogarden_amd.ds.sequence import Sequence
    from biogarden_amd.processing.patterns import (longest_common_subsequence,
                                                   shortest_common_supersequence)
    inp = read_fasta(os.path.join(REF_FIX, "input", "edit_distance.fasta"))
    assert edit_distance(Sequence(inp[0][1]), Sequence(inp[1][1])) == 299          # integration.rs:73
    assert edit_distance(Sequence("ACTGGATTC"), Sequence("ACGT")) == 5              # seq.rs:97-104
    inp = read_fasta(os.path.join(REF_FIX, "input", "longest_common_subseq.fasta"))
    out = read_fasta(os.path.join(REF_FIX, "output", "longest_common_subseq.fasta"))
    assert longest_common_subsequence(Sequence(inp[0][1]), Sequence(inp[1][1])) == Sequence(out[0][1])
    assert longest_common_subsequence(Sequence("AACCTTGG"), Sequence("ACACTGTGA")) == Sequence("ACCTGG")
    inp = read_fasta(os.path.join(REF_FIX, "input", "shortest_common_superseq.fasta"))
    out = read_fasta(os.path.join(REF_FIX, "output", "shortest_common_superseq.fasta"))
    assert shortest_common_supersequence(Sequence(inp[0][1]), Sequence(inp[1][1])) == Sequence(out[0][1])
    assert shortest_common_supersequence(Sequence("TGCATA"), Sequence("ATCTGAT")) == Sequence("ATGCATGAT")


@pytest.mark.parametrize("alpha", [DNA, PROT, b"AC", b"abcdefghijklmnopqrstuvwxyz0123-."])
def test_random_vs_oracle(oracle, alpha):
    from biogarden_amd.analysis.seq import edit_distance_batch
    from biogarden_amd.processing.patterns import (longest_common_subsequence_batch,
                                                   shortest_common_supersequence_batch)
    rng = random.Random(len(alpha))
    lens = [0, 1, 2, 5, 63, 64, 65, 130, 257, 600, 1100, 2300]
    pairs = []
    for _ in range(40):
        n1, n2 = rng.choice(lens), rng.choice(lens)
        s1 = rand_seq(rng, n1, alpha)
        s2 = mutate(rng, s1, alpha)[:n2] if rng.random() < 0.6 else rand_seq(rng, n2, alpha)
        pairs.append((s1, s2))
    got = edit_distance_batch(pairs)
    assert got == [oracle.edit_distance(a, b) for a, b in pairs]
    lcs = longest_common_subsequence_batch(pairs)
    assert [bytes(x.chain) for x in lcs] == [oracle.longest_common_subsequence(a, b) for a, b in pairs]
    scs = shortest_common_supersequence_batch(pairs)
    assert [bytes(x.chain) for x in scs] == [oracle.shortest_common_supersequence(a, b) for a, b in pairs]


def test_long_pairs(oracle):
    """Pairs spanning many strips and chunks (the recomputing traceback crosses strips)."""
    from biogarden_amd.analysis.seq import edit_distance_batch
    from biogarden_amd.processing.patterns import longest_common_subsequence_batch
    rng = random.Random(11)
    pairs = []
    for n1, n2 in ((5000, 4700), (3000, 6100), (4096, 4096)):
        s1 = rand_seq(rng, n1, DNA)
        pairs.append((s1, mutate(rng, s1, DNA, 0.3)[:n2]))
    assert edit_distance_batch(pairs) == [oracle.edit_distance(a, b) for a, b in pairs]
    assert [bytes(x.chain) for x in longest_common_subsequence_batch(pairs)] == \
        [oracle.longest_common_subsequence(a, b) for a, b in pairs]


@pytest.mark.parametrize("nsym", [33, 100, 256])
def test_wide_byte_alphabets_vs_oracle(oracle, nsym):
    """edit_distance / LCS / SCS over raw bytes (seq.rs:105-130, patterns.rs:82-118 compare bytes
    for equality: any of the 256 values) with more than 32 distinct bytes in the batch: the
    affine-family kernels with 8-bit codes (bg_batch_prepare_table's form)."""
    from biogarden_amd.analysis.seq import edit_distance, edit_distance_batch
    from biogarden_amd.processing.patterns import (longest_common_subsequence_batch,
                                                   shortest_common_supersequence_batch)
    rng = random.Random(nsym)
    alpha = bytes(rng.sample(range(256), nsym))
    pairs = []
    for n1, n2 in ((0, 5), (1, 1), (40, 40), (300, 280), (1500, 900), (64, 65), (2100, 2300)):
        s1 = rand_seq(rng, n1, alpha)
        s2 = mutate(rng, s1, alpha, 0.3)[:n2] if rng.random() < 0.7 else rand_seq(rng, n2, alpha)
        pairs.append((s1, s2))
    assert edit_distance_batch(pairs) == [oracle.edit_distance(a, b) for a, b in pairs]
    assert [bytes(x.chain) for x in longest_common_subsequence_batch(pairs)] == \
        [oracle.longest_common_subsequence(a, b) for a, b in pairs]
    assert [bytes(x.chain) for x in shortest_common_supersequence_batch(pairs)] == \
        [oracle.shortest_common_supersequence(a, b) for a, b in pairs]
    assert edit_distance(bytes(range(40)), bytes(range(40, 80))) == 40


@pytest.mark.parametrize("alpha", [DNA, PROT])
def test_lcs_beyond_checkpoint_chunk_keys(oracle, alpha):
    """LCS pairs whose seq2 spans >= 65536 chunks (> 4.19 M bytes) do not fit the recomputing
    traceback's chunk keys: they run the full-trace mask kernel with the LCS tie rule in its trace
    bits (patterns.rs:82-118, where bg_lcs_batch used to answer BG_E_SCORE_RANGE).  Bit-exact
    with the oracle, beside an ordinary pair in the same batch."""
    from biogarden_amd.processing.patterns import longest_common_subsequence_batch
    rng = random.Random(len(alpha) + 4)
    base = rand_seq(rng, 40, alpha)
    long2 = rand_seq(rng, 2_100_000, alpha) + mutate(rng, base, alpha, 0.2) + rand_seq(rng, 2_100_000, alpha)
    pairs = [(base, long2), (rand_seq(rng, 700, alpha), rand_seq(rng, 650, alpha))]
    got = [bytes(x.chain) for x in longest_common_subsequence_batch(pairs)]
    assert got == [oracle.longest_common_subsequence(a, b) for a, b in pairs]
