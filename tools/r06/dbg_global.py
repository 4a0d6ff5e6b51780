"""Round 6 diagnosis: the test_random_small global (-2, -2) batch under each DP plan (default,
WIDE off, SPAN off, fixed R / W), mismatches against the oracle per plan."""
import random, sys, zlib
sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
from test_gpu_parity import GAPS, rand_seq, mutate, DNA
from oracle import refcpu
from biogarden_amd import _native

mode, alpha, scoring = sys.argv[1] if len(sys.argv) > 1 else "global", DNA, "blosum62"
want = tuple(int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "-2,-2").split(","))
rng = random.Random(zlib.crc32(repr((mode, alpha, scoring)).encode()))
lens = [0, 1, 2, 3, 7, 31, 63, 64, 65, 100, 127, 128, 129, 200, 255, 256, 257, 300]
for a, b in GAPS:
    pairs = []
    for _ in range(24):
        n1, n2 = rng.choice(lens), rng.choice(lens)
        if mode == "fitting" and n1 < n2 and rng.random() < 0.8:
            n1, n2 = n2, n1
        s1 = rand_seq(rng, n1, alpha)
        s2 = mutate(rng, s1, alpha)[:n2] if rng.random() < 0.5 else rand_seq(rng, n2, alpha)
        pairs.append((s1, s2))
    if (a, b) == want:
        break
ref = [refcpu.align(mode, s1, s2, scoring, a, b, exact=True) for s1, s2 in pairs]
h = _native.Handle(0)
sc = _native.builtin_scoring(_native.BG_BLOSUM62)
for name, opts, tune in (("default", {}, (0, 0)), ("wide0", {"wide": 0}, (0, 0)),
                         ("wide0 span0", {"wide": 0, "span": 0}, (0, 0)),
                         ("R4 W1", {"wide": 0, "span": 0}, (4, 1)), ("R2 W4", {"wide": 0, "span": 0}, (2, 4))):
    for k in ("wide", "span"):
        h.set_option(k, None)
    for k, v in opts.items():
        h.set_option(k, v)
    h.set_tuning(*tune)
    got = h.align_batch(mode, pairs, sc, a, b)
    st = h.stats()
    bad = [(p, len(pairs[p][0]), len(pairs[p][1]), ref[p][1], got[p]["score"]) for p in range(len(pairs))
           if (got[p]["score"], got[p]["aligned1"], got[p]["aligned2"]) != ref[p][1:]]
    print(name, "R", st["R"], "W", st["waves"], "wide", st["wide"], "bad", len(bad), bad[:4], flush=True)
