# CPU study (not product code): do traceback paths from nearby cells of one row merge quickly?
# Decides whether speculative per-strip walks can start from a guessed entry.
# Coalescence of traceback paths (linear gaps, semiglobal M frame, tie priority Y > X > R) on
# random DNA with blosum62 -1/-2: from row r, start at the true path's column x and at x + d;
# follow m_trace pointers up; report after how many rows they meet.
import numpy as np, sys
rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
N = 3000
B = {('A','A'):4,('C','C'):9,('G','G'):6,('T','T'):5,('A','C'):0,('A','G'):0,('A','T'):0,('C','G'):-3,('C','T'):-1,('G','T'):-2}
S = np.zeros((4,4), dtype=np.int64)
L = "ACGT"
for (p,q),v in B.items():
    S[L.index(p),L.index(q)] = v; S[L.index(q),L.index(p)] = v
a = -1
s1 = rng.integers(0,4,N); s2 = rng.integers(0,4,N)
M = np.zeros((N+1,N+1), dtype=np.int64)
T = np.zeros((N+1,N+1), dtype=np.int8)   # 0 diag, 1 up, 2 left
for i in range(1,N+1):
    row = M[i-1]
    d = row[:-1] + S[s1[i-1], s2]
    x = row[1:] + a
    # y depends on left within the row: sequential
    Mi = M[i]
    Ti = T[i]
    for j in range(1,N+1):
        y = Mi[j-1] + a
        dd = d[j-1]; xx = x[j-1]
        best = max(dd, xx, y)
        Mi[j] = best
        Ti[j] = 2 if y == best else (1 if xx == best else 0)
    Ti[0] = 1
T[0,:] = 2
def walk(i, j, stop_row):
    path = {}
    while i > stop_row and i > 0 and j > 0:
        path.setdefault(i, j)
        t = T[i,j]
        if t == 0: i -= 1; j -= 1
        elif t == 1: i -= 1
        else: j -= 1
    return path
# true path from the bottom-right region
i0, j0 = N, int(np.argmax(M[N]))
true = walk(i0, j0, 0)
for r in (2800, 2000, 1200):
    x = true.get(r)
    if x is None: continue
    for dlt in (1, 5, 20, 100, 400):
        pa = walk(r, x, 0); pb = walk(r, min(N, x + dlt), 0)
        meet = None
        for row in range(r, 0, -1):
            if row in pa and row in pb and pa[row] == pb[row]:
                meet = r - row; break
        print(f"row {r} offset {dlt:4d}: merge after {meet} rows")
