"""Round 6: the self-serving traceback walker (round 5's one unexplained hang) repeated in ONE GPU
process: the test's batch under BG_FIN_SELFSERVE at 5 and 6 slots, R/W 8/16 and 2/4, N rounds,
every result against the oracle, no wait may run out (bg_wait_diag)."""
import random
import sys
import time

sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from parity_util import DNA, mutate, rand_seq
from oracle import refcpu
from biogarden_amd.alignment.aligner import SequenceAligner
from biogarden_amd.alignment import score

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
rng = random.Random(0x5E1F)
base = rand_seq(rng, 6000, DNA)
pairs = [(base, base[:3000] + rand_seq(rng, 3000, DNA) + base[3000:]),
         (base, base[:1500] + base[4000:]), (base, mutate(rng, base, DNA, 0.15)),
         (base, base), (base, mutate(rng, base, DNA, 0.01))]
expect = [refcpu.align("semiglobal", s1, s2, "blosum62", -1, -2, exact=True) for s1, s2 in pairs]
al = SequenceAligner()
t0 = time.time()
n = 0
for it in range(rounds):
    for slots in (5, 6):
        with al.options(fin_selfserve=1, fin_slots=slots):
            for R, W in ((8, 16), (2, 4)):
                al.set_tuning(R, W)
                res = al.align_batch("semiglobal", pairs, score.blosum62, -1, -2)
                assert al._h.wait_diag() is None, (it, slots, R, W, al._h.wait_diag())
                for e, r in zip(expect, res):
                    assert r.status in (0, 4), (it, slots, R, W, r.status)
                    assert (e[1], e[2], e[3]) == (r[0], bytes(r[1].chain), bytes(r[2].chain)), (it, slots, R, W)
                n += 1
    print("round", it, "ok", round(time.time() - t0, 1), "s", flush=True)
al.set_tuning(0, 0)
print("self-serve stress:", n, "batches, all strings equal, no wait ran out")
