"""Synthetic inputs of SURVEY.md §8(d)'s configurations (C1-C5, M), shared by bench.py,
tools/configs.py and the GPU parity tests, so all three see the same bytes.

Seed = 0xB10A11F0 + config index (M = 5); numpy's PCG64 is the portable PRNG.  DNA is i.i.d.
uniform over ACGT, protein over the 20 standard residues.  seq1 = rows, seq2 = columns, as in
the reference's *_alignment(seq1, seq2, ...) (aligner.rs:84, 150, 351).
"""
import numpy as np

DNA = np.frombuffer(b"ACGT", dtype=np.uint8)
PROT = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", dtype=np.uint8)
SEED0 = 0xB10A11F0

# (mode, scoring, open, extend) per config
PARAMS = {
    "C1": ("semiglobal", "blosum62", -1, -2),
    "C2": ("local", "blosum62", -11, -1),
    "C3": ("semiglobal", "blosum62", -1, -2),
    "C4": ("semiglobal", "blosum62", -1, -2),
    "C5": ("global", "blosum62", -11, -1),
    "M": ("semiglobal", "blosum62", -1, -2),
    # the metric's shape with a genuinely affine gap model (open < extend)
    "MA": ("semiglobal", "blosum62", -11, -1),
}


def rng_for(name, salt=0):
    idx = {"C1": 1, "C2": 2, "C3": 3, "C4": 4, "C5": 5, "M": 5, "MA": 6}[name]
    return np.random.default_rng(SEED0 + idx + salt)


def rand_seq(rng, alpha, n):
    return alpha[rng.integers(0, len(alpha), n)].tobytes()


def c2_pairs(npairs=1024, rng=None):
    """1024 pairs of independent uniform DNA, 1000 x 1000 (not 1024: len == 1024 panics a fresh
    reference aligner)."""
    rng = rng if rng is not None else rng_for("C2")
    return [(rand_seq(rng, DNA, 1000), rand_seq(rng, DNA, 1000)) for _ in range(npairs)]


def c3_pair(n=100000, rng=None):
    rng = rng if rng is not None else rng_for("C3")
    return [(rand_seq(rng, DNA, n), rand_seq(rng, DNA, n))]


def c4_pairs(nrefs=64, reads_per_ref=1024, read_len=150, ref_len=10000, sub=0.02, rng=None):
    """Reads (150 bp substrings at a uniform offset, 2 % substitutions) against 10 kbp refs;
    seq1 = read, seq2 = ref (the semiglobal row branch)."""
    rng = rng if rng is not None else rng_for("C4")
    refs = [rand_seq(rng, DNA, ref_len) for _ in range(nrefs)]
    pairs = []
    for r in refs:
        ra = np.frombuffer(r, dtype=np.uint8)
        for _ in range(reads_per_ref):
            o = int(rng.integers(0, ref_len - read_len))
            read = ra[o:o + read_len].copy()
            m = rng.random(read_len) < sub
            read[m] = DNA[rng.integers(0, 4, int(m.sum()))]
            pairs.append((read.tobytes(), r))
    return pairs


def c5_proteins(n=256, lo=64, hi=4000, rng=None):
    rng = rng if rng is not None else rng_for("C5")
    return [rand_seq(rng, PROT, int(rng.integers(lo, hi + 1))) for _ in range(n)]


def c5_pairs(rank=None, world=8):
    """All 32 640 unordered pairs (i < j, seq1 = i) of 256 proteins U[64, 4000]; with rank set,
    that rank's round-robin share of `world`."""
    prots = c5_proteins()
    allp = [(prots[i], prots[j]) for i in range(len(prots)) for j in range(i + 1, len(prots))]
    return allp if rank is None else allp[rank::world]


def metric_pairs(npairs=256, n1=10000, n2=10000, seed=None):
    """M: uniform DNA pairs, 10 000 x 10 000."""
    rng = np.random.default_rng(SEED0 + 5 if seed is None else seed)
    return [(rand_seq(rng, DNA, n1), rand_seq(rng, DNA, n2)) for _ in range(npairs)]


def cells(pairs):
    return sum(len(x) * len(y) for x, y in pairs)


# what each configuration is, for records
DESCRIPTION = {
    "C2": "1024 x (1000 x 1000) uniform DNA, local (Smith-Waterman) affine -11/-1, blosum62",
    "C3": "1 x (100 000 x 100 000) uniform DNA, semiglobal -1/-2, blosum62 (intra-pair tiling)",
    "C4": "65 536 reads (150 bp, 2 % substitutions) vs 64 refs of 10 kbp, semiglobal -1/-2, "
          "blosum62 (seq1 = read)",
    "C5": "all-vs-all of 256 proteins U[64, 4000] (32 640 pairs), global -11/-1, blosum62",
}


def job(name):
    """A whole configuration as one batch: (mode, pairs, open, extend)."""
    mode, _, a, b = PARAMS[name]
    if name == "C2":
        return mode, c2_pairs(), a, b
    if name == "C3":
        return mode, c3_pair(), a, b
    if name == "C4":
        return mode, c4_pairs(), a, b
    if name == "C5":
        return mode, c5_pairs(), a, b
    raise ValueError(name)
