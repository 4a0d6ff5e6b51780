import random, sys, tempfile, os
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from parity_util import DNA, mutate, rand_seq
from biogarden_amd.alignment import score
from biogarden_amd.alignment.aligner import SequenceAligner
from biogarden_amd.stream import AlignStream
handles = int(sys.argv[1])
rng = random.Random(handles)
refs = [rand_seq(rng, 3000, DNA) for _ in range(3)]
reads, which = [], []
for k in range(300):
    r = k % 3; o = rng.randint(0, 2800)
    reads.append(mutate(rng, refs[r][o:o + rng.randint(50, 200)], DNA, 0.04)); which.append(r)
pairs = [(reads[i], refs[which[i]]) for i in range(300)]
got = []
with AlignStream("semiglobal", score.blosum62, -1, -2, handles=handles) as st:
    for b in range(0, 300, 70):
        got += st.submit(pairs[b:b+70], tag=b)
    got += st.drain()
flat = [r for _, rs in got for r in rs]
al = SequenceAligner(0)
want = al.align_batch("semiglobal", pairs, score.blosum62, -1, -2)
bad = 0
for i, (g, w) in enumerate(zip(flat, want)):
    if (g.status, g[0], bytes(g[1].chain), bytes(g[2].chain), g.end) != (w.status, w[0], bytes(w[1].chain), bytes(w[2].chain), w.end):
        bad += 1
        if bad < 6:
            print(i, 'st', g.status, w.status, 'sc', g[0], w[0], 'end', g.end, w.end, 'start', g.start, w.start, 'len', len(g[1]), len(w[1]), 'eq1', bytes(g[1].chain)==bytes(w[1].chain), 'eq2', bytes(g[2].chain)==bytes(w[2].chain))
print('handles', handles, 'bad', bad)
