"""ctypes binding of the CPU oracle (oracle/liboracle.so).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the parity checker / timed CPU baseline.  See oracle/refcpu.h.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

MODES = {"global": 0, "local": 1, "fitting": 2, "overlap": 3, "semiglobal": 4}
STATUS = {0: "ok", 1: "InvalidArgumentRange", 2: "InvalidInputSize", 3: "panic(score)",
          4: "panic(index)", 5: "hang"}
BUILTIN = {"blosum62": 0, "pam250": 1, "unit": 2}


class OrScoring(ctypes.Structure):
    _fields_ = [("alphabet_size", ctypes.c_int32), ("code", ctypes.c_uint8 * 256),
                ("table", ctypes.c_int32 * 1024), ("wide_k", ctypes.c_int32),
                ("wide_code", ctypes.POINTER(ctypes.c_uint16)),
                ("wide_table", ctypes.POINTER(ctypes.c_int32))]


def wide_scoring(fn, symbols):
    """A closure S(byte1, byte2) tabulated over any byte set (up to 256 codes); bytes outside
    `symbols` panic."""
    syms = sorted(set(symbols))
    k = len(syms)
    code = (ctypes.c_uint16 * 256)(*([0xFFFF] * 256))
    for i, x in enumerate(syms):
        code[x] = i
    table = (ctypes.c_int32 * (k * k))()
    for i, x in enumerate(syms):
        for j, y in enumerate(syms):
            table[i * k + j] = int(fn(x, y))
    sc = OrScoring()
    sc.wide_k = k
    sc.wide_code = code
    sc.wide_table = table
    sc._keep = (code, table)
    return sc


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.or_aligner_new.restype = ctypes.c_void_p
        L.or_aligner_new_exact.restype = ctypes.c_void_p
        L.or_aligner_new_dims.restype = ctypes.c_void_p
        L.or_aligner_new_dims.argtypes = [ctypes.c_size_t, ctypes.c_size_t]
        L.or_aligner_free.argtypes = [ctypes.c_void_p]
        L.or_buffer_size.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.POINTER(ctypes.c_size_t)]
        L.or_scoring_builtin.argtypes = [ctypes.c_int, ctypes.POINTER(OrScoring)]
        L.or_align.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t,
                               ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(OrScoring),
                               ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                               ctypes.c_char_p, ctypes.c_char_p,
                               ctypes.POINTER(ctypes.c_size_t)]
        L.or_align.restype = ctypes.c_int
        L.or_align_batch.argtypes = [ctypes.c_int, ctypes.c_size_t,
                                     ctypes.POINTER(ctypes.c_char_p),
                                     ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.POINTER(ctypes.c_char_p),
                                     ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.POINTER(OrScoring), ctypes.c_int32, ctypes.c_int32,
                                     ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_int32),
                                     ctypes.POINTER(ctypes.c_int)]
        L.or_align_batch.restype = ctypes.c_double
        L.or_edit_distance.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                       ctypes.c_size_t]
        L.or_edit_distance.restype = ctypes.c_uint64
        L.or_lcs.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                             ctypes.c_char_p]
        L.or_lcs.restype = ctypes.c_size_t
        _LIB = L
    return _LIB


def scoring(name_or_table):
    """Built-in table by name, or a callable S(byte1, byte2) tabulated over 'A'..'Z'."""
    sc = OrScoring()
    if isinstance(name_or_table, str):
        lib().or_scoring_builtin(BUILTIN[name_or_table], ctypes.byref(sc))
    else:
        sc.alphabet_size = 26
        for b in range(256):
            sc.code[b] = (b - 65) if 65 <= b <= 90 else 0xFF
        for r in range(26):
            for c in range(26):
                sc.table[r * 32 + c] = int(name_or_table(65 + r, 65 + c))
    return sc


class Aligner:
    """Reference-faithful SequenceAligner (exact=False) or exact-size product semantics."""

    def __init__(self, exact=False, dims=None):
        L = lib()
        if dims is not None:
            self._p = L.or_aligner_new_dims(dims[0], dims[1])
        else:
            self._p = L.or_aligner_new_exact() if exact else L.or_aligner_new()

    def __del__(self):
        if getattr(self, "_p", None):
            lib().or_aligner_free(self._p)
            self._p = None

    def buffer_size(self):
        r, c = ctypes.c_size_t(), ctypes.c_size_t()
        lib().or_buffer_size(self._p, ctypes.byref(r), ctypes.byref(c))
        return r.value, c.value

    def align(self, mode, s1, s2, score="blosum62", a=-11, b=-1):
        """Returns (status, score, aligned1, aligned2)."""
        s1 = bytes(s1)
        s2 = bytes(s2)
        sc = score if isinstance(score, OrScoring) else scoring(score)
        cap = len(s1) + len(s2) + 1
        o1 = ctypes.create_string_buffer(cap)
        o2 = ctypes.create_string_buffer(cap)
        res = ctypes.c_int32()
        ln = ctypes.c_size_t()
        st = lib().or_align(self._p, MODES[mode], s1, len(s1), s2, len(s2), ctypes.byref(sc),
                            a, b, ctypes.byref(res), o1, o2, ctypes.byref(ln))
        return st, res.value, o1.raw[:ln.value], o2.raw[:ln.value]


def align(mode, s1, s2, score="blosum62", a=-11, b=-1, exact=False):
    return Aligner(exact).align(mode, s1, s2, score, a, b)


def align_batch(mode, pairs, score="blosum62", a=-11, b=-1, nthreads=1, exact=True):
    """Times the CPU baseline over `pairs` [(s1, s2)]; returns (seconds, scores, statuses)."""
    n = len(pairs)
    s1 = (ctypes.c_char_p * n)(*[bytes(p[0]) for p in pairs])
    s2 = (ctypes.c_char_p * n)(*[bytes(p[1]) for p in pairs])
    n1 = (ctypes.c_size_t * n)(*[len(p[0]) for p in pairs])
    n2 = (ctypes.c_size_t * n)(*[len(p[1]) for p in pairs])
    scores = (ctypes.c_int32 * n)()
    sts = (ctypes.c_int * n)()
    sc = score if isinstance(score, OrScoring) else scoring(score)
    secs = lib().or_align_batch(MODES[mode], n, s1, n1, s2, n2, ctypes.byref(sc), a, b,
                                nthreads, 1 if exact else 0, scores, sts)
    return secs, list(scores), list(sts)


def edit_distance(s1, s2):
    """analysis::seq::edit_distance (src/analysis/seq.rs:105-130)."""
    s1, s2 = bytes(s1), bytes(s2)
    return int(lib().or_edit_distance(s1, len(s1), s2, len(s2)))


def longest_common_subsequence(s1, s2):
    """processing::patterns::longest_common_subsequence (src/processing/patterns.rs:82-118)."""
    s1, s2 = bytes(s1), bytes(s2)
    out = ctypes.create_string_buffer(min(len(s1), len(s2)) + 1)
    n = lib().or_lcs(s1, len(s1), s2, len(s2), out)
    return out.raw[:n]


def shortest_common_supersequence(s1, s2):
    """processing::patterns::shortest_common_supersequence (src/processing/patterns.rs:198-235):
    interleave both sequences around their LCS."""
    lcs = longest_common_subsequence(s1, s2)
    it1, it2 = iter(bytes(s1)), iter(bytes(s2))
    out = bytearray()
    for c in lcs:
        for x in it1:
            if x == c:
                break
            out.append(x)
        for x in it2:
            if x == c:
                break
            out.append(x)
        out.append(c)
    out.extend(it1)
    out.extend(it2)
    return bytes(out)
