"""ctypes binding of libbiogarden_gpu.so (include/biogarden_gpu.h).

The product path: every alignment goes through this library's HIP kernels.  There is no CPU
fallback — if the library or a GPU is missing, calls raise NativeUnavailable.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libbiogarden_gpu.so")

BG_GLOBAL, BG_LOCAL, BG_FITTING, BG_OVERLAP, BG_SEMIGLOBAL = range(5)
MODES = {"global": BG_GLOBAL, "local": BG_LOCAL, "fitting": BG_FITTING,
         "overlap": BG_OVERLAP, "semiglobal": BG_SEMIGLOBAL}
BG_OK, BG_INVALID_ARGUMENT_RANGE, BG_INVALID_INPUT_SIZE, BG_UNSCORABLE, BG_REF_DIVERGENT, BG_INTERNAL = range(6)
BG_BLOSUM62, BG_PAM250, BG_UNIT = range(3)

# every symbol include/biogarden_gpu.h declares (checked by tests/test_abi.py)
EXPORTS = ["bg_scoring_builtin", "bg_aligner_new", "bg_aligner_free", "bg_align",
           "bg_align_batch", "bg_batch_prepare", "bg_batch_execute", "bg_batch_fetch",
           "bg_synchronize", "bg_get_stats", "bg_set_tuning", "bg_status_string",
           "bg_abi_version", "bg_profile_begin", "bg_profile_end", "bg_batch_export",
           "bg_set_pipeline", "bg_set_kernel_options", "bg_edit_distance_batch",
           "bg_lcs_batch", "bg_aligner_buffer_size", "bg_aligner_set_buffer_size",
           "bg_aligner_set_call_dims", "bg_host_timing", "bg_last_hip_error",
           "bg_batch_export_compact", "bg_compact_expand", "bg_fasta_open",
           "bg_batch_prepare_table", "bg_fasta_next_batch",
           "bg_fasta_close", "bg_split_stats", "bg_split_conc_diag", "bg_aligner_new_shared",
           "bg_set_async_fetch", "bg_group_new", "bg_group_free", "bg_group_size",
           "bg_group_member", "bg_group_align_batch", "bg_group_plan", "bg_group_buffer_size",
           "bg_group_timing", "bg_group_submit", "bg_group_collect", "bg_group_pending",
           "bg_get_stats_sized", "bg_batch_export_compact_bound", "bg_batch_export_compact_async",
           "bg_set_option", "bg_get_option", "bg_wait_diag"]

# bg_set_option keys (include/biogarden_gpu.h BG_OPT_*), by their BG_OPTIONS names
OPTIONS = ("grouped", "group_pairs", "group_waves", "wide_waves", "fin_waves", "fin_slots",
           "fin_sync", "fin_selfserve", "split", "split_segment", "split_concurrent",
           "split_wait_ms", "two_dp_streams", "wait_ms", "span", "wide")


class NativeUnavailable(RuntimeError):
    pass


class BgScoring(ctypes.Structure):
    _fields_ = [("alphabet_size", ctypes.c_int32), ("code", ctypes.c_uint8 * 256),
                ("table", ctypes.c_int32 * 1024)]


class WideScoring:
    """A score table over up to 256 codes (bg_batch_prepare_table): code[byte] (>= k: the
    closure panics on that byte) and a k x k table, row = seq1 code."""

    def __init__(self, code, k, table):
        self.code = (ctypes.c_uint16 * 256)(*code)
        self.k = k
        self.table = (ctypes.c_int32 * (k * k))(*table)


class BgPairResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("score", ctypes.c_int32),
                ("offset", ctypes.c_uint64), ("len", ctypes.c_uint32),
                ("end_i", ctypes.c_uint32), ("end_j", ctypes.c_uint32),
                ("start1", ctypes.c_uint32), ("start2", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


class BgStats(ctypes.Structure):
    _fields_ = [("cells", ctypes.c_uint64), ("trace_bytes", ctypes.c_uint64),
                ("boundary_bytes", ctypes.c_uint64), ("residue_bytes", ctypes.c_uint64),
                ("device_bytes", ctypes.c_uint64), ("R", ctypes.c_int32),
                ("waves", ctypes.c_int32), ("affine", ctypes.c_int32), ("tagged", ctypes.c_int32),
                ("dna", ctypes.c_int32),
                ("local", ctypes.c_int32), ("npairs", ctypes.c_int32),
                ("wide", ctypes.c_int32), ("workgroups", ctypes.c_int32),
                ("checkpoint", ctypes.c_int32),
                ("dp_ms", ctypes.c_float), ("finish_ms", ctypes.c_float),
                ("fin_waves", ctypes.c_int32), ("fin_slots", ctypes.c_int32),
                ("split", ctypes.c_int32), ("grouped", ctypes.c_int32),
                ("group_pairs", ctypes.c_int32)]


class BgFastaBatch(ctypes.Structure):
    _fields_ = [("n", ctypes.c_size_t), ("seq", ctypes.c_void_p),
                ("seq_off", ctypes.POINTER(ctypes.c_uint64)), ("text", ctypes.c_void_p),
                ("id_off", ctypes.POINTER(ctypes.c_uint64)),
                ("desc_off", ctypes.POINTER(ctypes.c_uint64))]


_LIB = None


def lib():
    """Loads the HIP library; raises NativeUnavailable when it is not built."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise NativeUnavailable(
            "libbiogarden_gpu.so is not built (run __graft_entry__.build() or make -C "
            "biogarden_amd/csrc)")
    L = ctypes.CDLL(LIB_PATH)
    c_u8p = ctypes.POINTER(ctypes.c_uint8)
    L.bg_scoring_builtin.argtypes = [ctypes.c_int, ctypes.POINTER(BgScoring)]
    L.bg_aligner_new.argtypes = [ctypes.c_int]
    L.bg_aligner_new.restype = ctypes.c_void_p
    L.bg_aligner_new_shared.argtypes = [ctypes.c_void_p]
    L.bg_aligner_new_shared.restype = ctypes.c_void_p
    L.bg_set_async_fetch.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.bg_aligner_free.argtypes = [ctypes.c_void_p]
    L.bg_aligner_free.restype = None
    L.bg_align.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t,
                           ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(BgScoring),
                           ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                           ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
                           ctypes.POINTER(ctypes.c_size_t)]
    batch_args = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t,
                  ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                  ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                  ctypes.POINTER(BgScoring), ctypes.c_int32, ctypes.c_int32]
    L.bg_align_batch.argtypes = batch_args + [ctypes.POINTER(BgPairResult), c_u8p, c_u8p,
                                              ctypes.c_size_t]
    L.bg_batch_prepare.argtypes = batch_args
    L.bg_batch_prepare_table.argtypes = batch_args[:7] + [
        ctypes.POINTER(ctypes.c_uint16), ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
        ctypes.c_int32, ctypes.c_int32]
    L.bg_batch_execute.argtypes = [ctypes.c_void_p]
    L.bg_synchronize.argtypes = [ctypes.c_void_p]
    L.bg_batch_fetch.argtypes = [ctypes.c_void_p, ctypes.POINTER(BgPairResult), c_u8p, c_u8p,
                                 ctypes.c_size_t]
    L.bg_get_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(BgStats)]
    L.bg_get_stats_sized.argtypes = [ctypes.c_void_p, ctypes.POINTER(BgStats), ctypes.c_size_t]
    L.bg_split_stats.argtypes = [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_uint64)] * 5
    L.bg_split_conc_diag.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]
    L.bg_aligner_buffer_size.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                                         ctypes.POINTER(ctypes.c_size_t)]
    L.bg_aligner_set_buffer_size.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t]
    L.bg_aligner_set_call_dims.argtypes = [ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.POINTER(ctypes.c_uint64)]
    L.bg_set_tuning.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    L.bg_set_pipeline.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.bg_set_kernel_options.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.bg_set_option.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    L.bg_get_option.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    L.bg_wait_diag.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t]
    L.bg_status_string.argtypes = [ctypes.c_int]
    L.bg_status_string.restype = ctypes.c_char_p
    L.bg_abi_version.restype = ctypes.c_int
    L.bg_profile_begin.argtypes = [ctypes.c_void_p]
    L.bg_profile_end.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float),
                                 ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)]
    L.bg_batch_export_compact.argtypes = [ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.POINTER(ctypes.c_size_t)]
    L.bg_batch_export_compact_bound.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t)]
    L.bg_batch_export_compact_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                ctypes.c_void_p]
    L.bg_compact_expand.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                    ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                    ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                    ctypes.POINTER(BgPairResult), c_u8p, c_u8p, ctypes.c_size_t]
    L.bg_host_timing.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_size_t,
                                 ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    L.bg_batch_export.argtypes = [ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.POINTER(ctypes.c_size_t)]
    pair_args = [ctypes.c_void_p, ctypes.c_size_t,
                 ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                 ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t)]
    L.bg_edit_distance_batch.argtypes = pair_args + [ctypes.POINTER(ctypes.c_uint64)]
    L.bg_lcs_batch.argtypes = pair_args + [c_u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.POINTER(ctypes.c_uint64)]
    L.bg_group_new.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    L.bg_group_new.restype = ctypes.c_void_p
    L.bg_group_free.argtypes = [ctypes.c_void_p]
    L.bg_group_free.restype = None
    L.bg_group_size.argtypes = [ctypes.c_void_p]
    L.bg_group_member.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.bg_group_member.restype = ctypes.c_void_p
    L.bg_group_align_batch.argtypes = [ctypes.c_void_p] + batch_args[1:] + [
        ctypes.POINTER(BgPairResult), c_u8p, c_u8p, ctypes.c_size_t]
    L.bg_group_submit.argtypes = [ctypes.c_void_p] + batch_args[1:]
    L.bg_group_collect.argtypes = [ctypes.c_void_p, ctypes.POINTER(BgPairResult), c_u8p, c_u8p,
                                   ctypes.c_size_t]
    L.bg_group_pending.argtypes = [ctypes.c_void_p]
    L.bg_group_plan.argtypes = [ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                                ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
                                ctypes.POINTER(ctypes.c_int32)]
    L.bg_group_buffer_size.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                                       ctypes.POINTER(ctypes.c_size_t)]
    L.bg_group_timing.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_size_t,
                                  ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    L.bg_fasta_open.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
    L.bg_fasta_open.restype = ctypes.c_void_p
    L.bg_fasta_next_batch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                      ctypes.POINTER(BgFastaBatch)]
    L.bg_fasta_next_batch.restype = ctypes.c_long
    L.bg_fasta_close.argtypes = [ctypes.c_void_p]
    L.bg_fasta_close.restype = None
    _LIB = L
    return L


def builtin_scoring(which):
    sc = BgScoring()
    rc = lib().bg_scoring_builtin(which, ctypes.byref(sc))
    if rc != 0:
        raise ValueError("unknown built-in table %r" % which)
    return sc


def check(rc):
    if rc < 0:
        msg = "biogarden_gpu: %s (%d)" % (lib().bg_status_string(rc).decode(), rc)
        if rc == -2:
            msg += ", hipError_t %d" % lib().bg_last_hip_error()
        raise RuntimeError(msg)
    return rc


class Handle:
    """One bg_aligner (device scratch arenas + HIP streams) on one GPU.  share=<Handle>: a handle
    on the same GPU that shares that handle's HIP streams (bg_aligner_new_shared)."""

    def __init__(self, device=0, share=None):
        if share is not None:
            self._p = lib().bg_aligner_new_shared(share._p)
            device = share.device
        else:
            self._p = lib().bg_aligner_new(int(device))
        if not self._p:
            raise NativeUnavailable("bg_aligner_new(%d) failed: no usable HIP device" % device)
        self.device = device

    def close(self):
        if getattr(self, "_p", None):
            lib().bg_aligner_free(self._p)
            self._p = None

    __del__ = close

    def set_tuning(self, R=0, waves=0):
        check(lib().bg_set_tuning(self._p, R, waves))

    def set_kernel_options(self, allow_tagged=True, checkpoint=True, affine_checkpoint=True):
        """allow_tagged: tagged linear kernel (else mask trace); checkpoint: score-only DP with
        the traceback recomputing the chunks it crosses (else the full trace is written);
        affine_checkpoint: the same for affine gaps / local mode / > 4 symbols (else the
        mask-trace kernel)."""
        check(lib().bg_set_kernel_options(self._p, (1 if allow_tagged else 0) |
                                          (2 if (allow_tagged and checkpoint) else 0) |
                                          (4 if affine_checkpoint else 0)))

    def set_option(self, name, value):
        """bg_set_option by name (OPTIONS); value None or -1 restores the automatic choice."""
        check(lib().bg_set_option(self._p, OPTIONS.index(name), -1 if value is None else int(value)))

    def get_option(self, name):
        v = ctypes.c_int()
        check(lib().bg_get_option(self._p, OPTIONS.index(name), ctypes.byref(v)))
        return v.value

    def options(self, **kw):
        """Context manager: set options for a block, restore the previous values after it."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            old = {k: self.get_option(k) for k in kw}
            try:
                for k, v in kw.items():
                    self.set_option(k, v)
                yield self
            finally:
                for k, v in old.items():
                    self.set_option(k, v)
        return cm()

    def set_pipeline(self, depth):
        check(lib().bg_set_pipeline(self._p, depth))

    def set_async_fetch(self, on=True):
        """bg_set_async_fetch: every execute queues its results' download behind its traceback;
        fetch() then only waits and unpacks."""
        check(lib().bg_set_async_fetch(self._p, 1 if on else 0))

    @staticmethod
    def _arrays(pairs):
        n = len(pairs)
        s1 = [bytes(p[0]) for p in pairs]
        s2 = [bytes(p[1]) for p in pairs]
        a1 = (ctypes.c_char_p * n)(*s1)
        a2 = (ctypes.c_char_p * n)(*s2)
        n1 = (ctypes.c_size_t * n)(*[len(x) for x in s1])
        n2 = (ctypes.c_size_t * n)(*[len(x) for x in s2])
        return a1, n1, a2, n2, sum(len(x) for x in s1) + sum(len(x) for x in s2)

    @staticmethod
    def _packed_arrays(buf1, off1, idx1, buf2, off2, idx2):
        """Pointer + length arrays into two packed residue buffers (bytes objects, e.g. FASTA
        batches): pair p is buf1[off1[idx1[p]]:off1[idx1[p]+1]] against the same in buf2.
        No per-pair copy."""
        import numpy as np
        n = len(idx1)
        b1 = ctypes.cast(ctypes.c_char_p(buf1), ctypes.c_void_p).value or 0
        b2 = ctypes.cast(ctypes.c_char_p(buf2), ctypes.c_void_p).value or 0
        o1, o2 = np.asarray(off1, dtype=np.uint64), np.asarray(off2, dtype=np.uint64)
        i1, i2 = np.asarray(idx1, dtype=np.int64), np.asarray(idx2, dtype=np.int64)
        p1 = (np.uint64(b1) + o1[i1]).astype(np.uint64)
        p2 = (np.uint64(b2) + o2[i2]).astype(np.uint64)
        l1 = (o1[i1 + 1] - o1[i1]).astype(np.uint64)
        l2 = (o2[i2 + 1] - o2[i2]).astype(np.uint64)
        a1 = (ctypes.c_uint64 * max(n, 1)).from_buffer_copy(p1.tobytes() or bytes(8))
        a2 = (ctypes.c_uint64 * max(n, 1)).from_buffer_copy(p2.tobytes() or bytes(8))
        n1 = (ctypes.c_size_t * max(n, 1)).from_buffer_copy(l1.tobytes() or bytes(8))
        n2 = (ctypes.c_size_t * max(n, 1)).from_buffer_copy(l2.tobytes() or bytes(8))
        return (ctypes.cast(a1, ctypes.POINTER(ctypes.c_char_p)), n1,
                ctypes.cast(a2, ctypes.POINTER(ctypes.c_char_p)), n2,
                int(l1.sum()) + int(l2.sum()), (buf1, buf2, a1, a2))

    def prepare_packed(self, mode, buf1, off1, idx1, buf2, off2, idx2, scoring, a, b):
        """prepare() for pairs given as indices into two packed residue buffers."""
        a1, n1, a2, n2, total, keep = self._packed_arrays(buf1, off1, idx1, buf2, off2, idx2)
        self._keep = (a1, n1, a2, n2, keep)
        self._npairs = len(idx1)
        self._total = total
        check(self._prepare_call(mode, len(idx1), a1, n1, a2, n2, scoring, a, b))

    def _prepare_call(self, mode, n, a1, n1, a2, n2, scoring, a, b):
        if isinstance(scoring, WideScoring):
            return lib().bg_batch_prepare_table(self._p, MODES.get(mode, mode), n, a1, n1, a2, n2,
                                                scoring.code, scoring.k, scoring.table, a, b)
        return lib().bg_batch_prepare(self._p, MODES.get(mode, mode), n, a1, n1, a2, n2,
                                      ctypes.byref(scoring), a, b)

    def prepare(self, mode, pairs, scoring, a, b):
        a1, n1, a2, n2, total = self._arrays(pairs)
        self._keep = (a1, n1, a2, n2)
        self._npairs = len(pairs)
        self._total = total
        check(self._prepare_call(mode, len(pairs), a1, n1, a2, n2, scoring, a, b))

    def execute(self):
        check(lib().bg_batch_execute(self._p))

    def synchronize(self):
        check(lib().bg_synchronize(self._p))

    def fetch(self):
        n = self._npairs
        res = (BgPairResult * max(n, 1))()
        o1 = (ctypes.c_uint8 * max(self._total, 1))()
        o2 = (ctypes.c_uint8 * max(self._total, 1))()
        check(lib().bg_batch_fetch(self._p, res, o1, o2, self._total))
        b1 = bytes(o1)
        b2 = bytes(o2)
        out = []
        for p in range(n):
            r = res[p]
            lo, hi = r.offset, r.offset + r.len
            out.append({"status": r.status, "score": r.score, "aligned1": b1[lo:hi],
                        "aligned2": b2[lo:hi], "end": (r.end_i, r.end_j),
                        "start": (r.start1, r.start2)})
        return out

    def fetch_raw(self):
        """bg_batch_fetch into handle-owned ctypes buffers, without per-pair Python objects:
        {"status": [..], "score": [..], "offset": [..], "len": [..], "out1": buf, "out2": buf}
        (the buffers are reused by the next fetch_raw)."""
        n = self._npairs
        need = max(self._total, 1)
        if getattr(self, "_raw_cap", 0) < need or getattr(self, "_raw_n", 0) < max(n, 1):
            self._raw_res = (BgPairResult * max(n, 1))()
            self._raw_o1 = (ctypes.c_uint8 * need)()
            self._raw_o2 = (ctypes.c_uint8 * need)()
            self._raw_cap = need
            self._raw_n = max(n, 1)
        check(lib().bg_batch_fetch(self._p, self._raw_res, self._raw_o1, self._raw_o2, self._total))
        res = self._raw_res
        return {"status": [res[p].status for p in range(n)],
                "score": [res[p].score for p in range(n)],
                "offset": [res[p].offset for p in range(n)],
                "len": [res[p].len for p in range(n)],
                "out1": self._raw_o1, "out2": self._raw_o2}

    def align_batch(self, mode, pairs, scoring, a, b):
        self.prepare(mode, pairs, scoring, a, b)
        self.execute()
        return self.fetch()

    def profile_begin(self):
        check(lib().bg_profile_begin(self._p))

    def profile_end(self):
        """-> (avg DP kernel ms, avg finish kernel ms, executes) over the profiled region."""
        dp, fin, n = ctypes.c_float(), ctypes.c_float(), ctypes.c_int()
        check(lib().bg_profile_end(self._p, ctypes.byref(dp), ctypes.byref(fin), ctypes.byref(n)))
        return dp.value, fin.value, n.value

    def export_size(self):
        n = ctypes.c_size_t(0)
        check(lib().bg_batch_export(self._p, None, ctypes.byref(n)))
        return n.value

    def export_to(self, device_ptr, nbytes):
        """Packs the last execute's results into device memory at device_ptr (same GPU)."""
        n = ctypes.c_size_t(nbytes)
        check(lib().bg_batch_export(self._p, ctypes.c_void_p(device_ptr), ctypes.byref(n)))
        return n.value

    def export_compact_size(self):
        """Bytes of the compact export record of the last execute (computes it on the device)."""
        n = ctypes.c_size_t(0)
        check(lib().bg_batch_export_compact(self._p, None, ctypes.byref(n)))
        return n.value

    def export_compact_to(self, device_ptr, nbytes):
        """Writes the compact record (bg_batch_export_compact) to device memory of this GPU."""
        n = ctypes.c_size_t(nbytes)
        check(lib().bg_batch_export_compact(self._p, ctypes.c_void_p(device_ptr), ctypes.byref(n)))
        return n.value

    def export_compact_bound(self):
        """The compact record's largest size for the prepared batch (no device work)."""
        n = ctypes.c_size_t(0)
        check(lib().bg_batch_export_compact_bound(self._p, ctypes.byref(n)))
        return n.value

    def export_compact_async(self, device_ptr, cap, after_stream=None):
        """bg_batch_export_compact_async: the last execute's compact record into device memory
        without a host wait; after_stream (a raw hipStream_t, e.g. torch's current stream's
        cuda_stream; 0 / None = the null stream) waits for it."""
        check(lib().bg_batch_export_compact_async(self._p, ctypes.c_void_p(device_ptr), cap,
                                                  ctypes.c_void_p(after_stream or 0)))

    def edit_distance_batch(self, pairs):
        """analysis::seq::edit_distance over pairs [(s1, s2)] -> [int]."""
        a1, n1, a2, n2, _ = self._arrays(pairs)
        n = len(pairs)
        out = (ctypes.c_uint64 * max(n, 1))()
        check(lib().bg_edit_distance_batch(self._p, n, a1, n1, a2, n2, out))
        return [int(out[p]) for p in range(n)]

    def lcs_batch(self, pairs):
        """processing::patterns::longest_common_subsequence over pairs -> [bytes]."""
        a1, n1, a2, n2, _ = self._arrays(pairs)
        n = len(pairs)
        cap = max(1, sum(min(len(x), len(y)) for x, y in pairs))
        buf = (ctypes.c_uint8 * cap)()
        off = (ctypes.c_uint64 * max(n, 1))()
        ln = (ctypes.c_uint64 * max(n, 1))()
        check(lib().bg_lcs_batch(self._p, n, a1, n1, a2, n2, buf, cap, off, ln))
        raw = bytes(buf)
        return [raw[off[p]:off[p] + ln[p]] for p in range(n)]

    def buffer_size(self):
        """The reference aligner's scratch dims this handle models (aligner.rs:30)."""
        r, c = ctypes.c_size_t(), ctypes.c_size_t()
        check(lib().bg_aligner_buffer_size(self._p, ctypes.byref(r), ctypes.byref(c)))
        return r.value, c.value

    def set_buffer_size(self, rows, cols):
        check(lib().bg_aligner_set_buffer_size(self._p, rows, cols))

    def set_call_dims(self, dims):
        """Per-pair scratch dims the next prepared batch's calls start from (a shard of a larger
        batch: shard.call_dims); None or [] clears."""
        n = len(dims) if dims else 0
        rows = (ctypes.c_uint64 * max(n, 1))(*[d[0] for d in dims or []])
        cols = (ctypes.c_uint64 * max(n, 1))(*[d[1] for d in dims or []])
        check(lib().bg_aligner_set_call_dims(self._p, n, rows, cols))

    HOST_PHASES = ("wait_previous", "validate_stage", "plan", "alloc", "upload", "fetch_wait",
                   "fetch_d2h", "fetch_unpack")

    def host_timing(self, reset=False):
        """Accumulated host-side ms per phase of prepare / fetch (bg_host_timing), plus the call
        counts and the host threads of the byte passes."""
        ms = (ctypes.c_double * 8)()
        calls = (ctypes.c_uint64 * 3)()
        check(lib().bg_host_timing(self._p, ms, 8, calls, 1 if reset else 0))
        out = {k: ms[i] for i, k in enumerate(self.HOST_PHASES)}
        out.update({"prepares": calls[0], "fetches": calls[1], "host_threads": calls[2]})
        return out

    def stats(self):
        st = BgStats()
        check(lib().bg_get_stats_sized(self._p, ctypes.byref(st), ctypes.sizeof(st)))
        return {f: getattr(st, f) for f, _ in BgStats._fields_}

    def split_stats(self):
        """bg_split_stats: the last execute's split traceback (pairs split, strips stitched,
        moves the stitching walked itself, pairs whose exit pass overflowed)."""
        v = [ctypes.c_uint64() for _ in range(5)]
        check(lib().bg_split_stats(self._p, *[ctypes.byref(x) for x in v]))
        return dict(zip(("pairs_split", "strips_taken", "tail_moves", "pairs_overflow", "items_beside_dp"),
                        (x.value for x in v)))

    WAIT_KINDS = {0: None, 1: "walker waited for a chunk", 2: "walker waited for the slot lock",
                  3: "helper waited for the slot lock", 4: "walker recomputed one chunk over and over"}

    def wait_diag(self):
        """bg_wait_diag: the last execute's traceback wait that ran out (None if none did)."""
        v = (ctypes.c_uint32 * 18)()
        check(lib().bg_wait_diag(self._p, v, 18))
        if v[0] == 0:
            return None
        return {"kind": self.WAIT_KINDS.get(v[0], v[0]), "pair": v[1], "wave": v[2],
                "key": (v[3] >> 16, v[3] & 0xFFFF), "map": v[4], "filling": v[5], "lock": v[6],
                "walker": (v[7], v[8]), "recomputed": v[9], "slots": list(v[10:18])}

    def conc_diag(self):
        """bg_split_conc_diag: the concurrent exit pass's abandon record (all zero: it ran to
        the end of its items, or was not used)."""
        v = (ctypes.c_uint32 * 6)()
        check(lib().bg_split_conc_diag(self._p, v))
        return dict(zip(("abandoned", "item", "input", "tag_seen", "epoch", "not_resident"), list(v)))


class Group:
    """bg_group: one process driving several GPUs (a device may repeat: several shards on one
    GPU).  align_batch splits the pairs over the members by cells, aligns every shard on its
    device, gathers the compact records to the first member's device over RCCL and expands them
    on the host — the same results as Handle.align_batch on one aligner."""

    PHASES = ("prepare_execute", "export", "gather", "download", "expand")

    def __init__(self, devices):
        devs = (ctypes.c_int * len(devices))(*devices)
        self._p = lib().bg_group_new(devs, len(devices))
        if not self._p:
            raise NativeUnavailable("bg_group_new(%r) failed (no such device, or no librccl)"
                                    % (list(devices),))
        self.devices = list(devices)
        self._tickets = []          # submitted, not yet collected (bg_group_collect takes the oldest)

    def close(self):
        if getattr(self, "_p", None):
            lib().bg_group_free(self._p)
            self._p = None

    __del__ = close

    def __len__(self):
        return lib().bg_group_size(self._p)

    def align_batch_raw(self, mode, pairs, scoring, a, b):
        """-> (results ctypes array, out1, out2) without per-pair Python objects."""
        a1, n1, a2, n2, total = Handle._arrays(pairs)
        n = len(pairs)
        res = (BgPairResult * max(n, 1))()
        o1 = (ctypes.c_uint8 * max(total, 1))()
        o2 = (ctypes.c_uint8 * max(total, 1))()
        check(lib().bg_group_align_batch(self._p, MODES.get(mode, mode), n, a1, n1, a2, n2,
                                         ctypes.byref(scoring), a, b, res, o1, o2, total))
        return res, o1, o2

    def align_batch(self, mode, pairs, scoring, a, b):
        res, o1, o2 = self.align_batch_raw(mode, pairs, scoring, a, b)
        b1, b2 = bytes(o1), bytes(o2)
        out = []
        for p in range(len(pairs)):
            r = res[p]
            lo, hi = r.offset, r.offset + r.len
            out.append({"status": r.status, "score": r.score, "aligned1": b1[lo:hi],
                        "aligned2": b2[lo:hi], "end": (r.end_i, r.end_j),
                        "start": (r.start1, r.start2)})
        return out

    def submit(self, mode, pairs, scoring, a, b):
        """bg_group_submit: queue one batch (at most three in flight); returns a ticket that
        collect() consumes in submission order.  The ticket holds the sequence buffers alive."""
        a1, n1, a2, n2, total = Handle._arrays(pairs)
        check(lib().bg_group_submit(self._p, MODES.get(mode, mode), len(pairs), a1, n1, a2, n2,
                                    ctypes.byref(scoring), a, b))
        ticket = (a1, n1, a2, n2, total, len(pairs), pairs)
        self._tickets.append(ticket)
        return ticket

    def collect(self, ticket, bufs=None):
        """bg_group_collect for the oldest submitted batch (pass its ticket): -> (results, out1,
        out2) as align_batch_raw.  bufs: a (results, out1, out2) triple to reuse, as large as the
        batch needs (a streaming caller rotates a few; fresh buffers fault their pages in)."""
        # bg_group_collect always finishes the OLDEST batch and writes that batch's pair count of
        # results: any other ticket would size the buffers for the wrong batch
        if self._tickets and ticket is not self._tickets[0]:
            raise ValueError("collect() takes the oldest submitted ticket (submission order)")
        total, n = ticket[4], ticket[5]
        if bufs is not None and len(bufs[0]) >= n and len(bufs[1]) >= total and len(bufs[2]) >= total:
            res, o1, o2 = bufs
        else:
            res = (BgPairResult * max(n, 1))()
            o1 = (ctypes.c_uint8 * max(total, 1))()
            o2 = (ctypes.c_uint8 * max(total, 1))()
        check(lib().bg_group_collect(self._p, res, o1, o2, max(total, 1) if bufs is None else len(o1)))
        if self._tickets:
            self._tickets.pop(0)
        return res, o1, o2

    def pending(self):
        return lib().bg_group_pending(self._p)

    def buffer_size(self):
        r, c = ctypes.c_size_t(), ctypes.c_size_t()
        check(lib().bg_group_buffer_size(self._p, ctypes.byref(r), ctypes.byref(c)))
        return r.value, c.value

    def timing(self, reset=False):
        ms = (ctypes.c_double * 5)()
        calls = ctypes.c_uint64()
        check(lib().bg_group_timing(self._p, ms, 5, ctypes.byref(calls), 1 if reset else 0))
        out = {k: ms[i] for i, k in enumerate(self.PHASES)}
        out["calls"] = calls.value
        return out


def group_plan(sizes, nshards):
    """bg_group_plan (host only): the member of every pair, [(n1, n2)] -> [int]."""
    n = len(sizes)
    n1 = (ctypes.c_size_t * max(n, 1))(*[x for x, _ in sizes])
    n2 = (ctypes.c_size_t * max(n, 1))(*[y for _, y in sizes])
    out = (ctypes.c_int32 * max(n, 1))()
    check(lib().bg_group_plan(n, n1, n2, nshards, out))
    return [out[p] for p in range(n)]


def expand_compact(rec, pairs):
    """bg_compact_expand: a compact export record (bytes) of `pairs` [(s1, s2)] -> the result
    dicts bg_batch_fetch gives for them (status, score, both aligned strings, end, start)."""
    rec = bytes(rec)
    a1, n1, a2, n2, total = Handle._arrays(pairs)
    n = len(pairs)
    res = (BgPairResult * max(n, 1))()
    o1 = (ctypes.c_uint8 * max(total, 1))()
    o2 = (ctypes.c_uint8 * max(total, 1))()
    check(lib().bg_compact_expand(rec, len(rec), n, a1, n1, a2, n2, res, o1, o2, total))
    b1, b2 = bytes(o1), bytes(o2)
    out = []
    for p in range(n):
        r = res[p]
        lo, hi = r.offset, r.offset + r.len
        out.append({"status": r.status, "score": r.score, "aligned1": b1[lo:hi], "aligned2": b2[lo:hi],
                    "end": (r.end_i, r.end_j), "start": (r.start1, r.start2)})
    return out


def compact_headers(rec):
    """The per-pair (status, score, len) of a compact export record, without expanding strings."""
    import struct
    rec = bytes(rec)
    magic, n, _ops, _mode = struct.unpack_from("<4Q", rec, 0)
    if magic != 0x31434742:
        raise ValueError("not a compact export record")
    out = []
    for p in range(n):
        st, sc, _off, ln = struct.unpack_from("<iiQI", rec, 32 + 48 * p)
        out.append((st, sc, ln))
    return out


def decode_export(buf):
    """Parses a bg_batch_export record (bytes) -> list of result dicts (for rank 0 after a
    gather)."""
    import struct
    n = struct.unpack_from("<Q", buf, 0)[0]
    rs = ctypes.sizeof(BgPairResult)
    recs = [BgPairResult.from_buffer_copy(buf, 8 + i * rs) for i in range(n)]
    base1 = 8 + n * rs
    out_bytes = (len(buf) - base1) // 2
    base2 = base1 + out_bytes
    out = []
    for r in recs:
        out.append({"status": r.status, "score": r.score,
                    "aligned1": bytes(buf[base1 + r.offset: base1 + r.offset + r.len]),
                    "aligned2": bytes(buf[base2 + r.offset: base2 + r.offset + r.len]),
                    "end": (r.end_i, r.end_j), "start": (r.start1, r.start2)})
    return out
