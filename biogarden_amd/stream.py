"""Streaming batch alignment on one GPU: FASTA -> packed residues -> HBM, overlapped with the
kernels.

`AlignStream` keeps a rotation of handles (`bg_aligner`, each with its own arenas and batch).
Submitting batch k stages its residues in pinned memory and queues its upload and kernels on
handle k mod H while batches k-1 .. k-H+1 are still on the GPU; the oldest batch is collected
(its aligned strings unpacked into host buffers) only when its handle comes round again.

The handles share ONE set of HIP streams (`bg_aligner_new_shared`): uploads, DPs, tracebacks and
downloads, four hardware queues in all, so no copy waits in a queue behind another batch's
kernel (the MI355X boxes give a process 4 queues, GPU_MAX_HW_QUEUES).  The DPs of consecutive
batches run back to back on the DP stream with each traceback beside the next DP, as one
handle's executes do, and every execute queues its strings' download right behind its traceback
(`bg_set_async_fetch`).  The host's byte passes, the PCIe copies and the kernels of different
batches therefore overlap, and the GPU sees a steady queue of batches (bench.py's
`host_to_host` leg measures it).

    with AlignStream("semiglobal", score.blosum62, -1, -2) as st:
        for reads in fasta.BatchReader("reads.fa", max_records=8192):
            for tag, results in st.submit(pairs_for(reads), tag=...):
                consume(tag, results)
        for tag, results in st.drain():
            consume(tag, results)

Each result is the AlignmentResult of SequenceAligner.align_batch (score, aligned seq1,
aligned seq2, .status, .end, .start).  Results come back in submission order.  The stream
stands for ONE reference aligner: the scratch dims that decide the reference-divergence flag
(status 4, aligner.rs:92-94) pass from handle to handle in submission order, so a stream
flags exactly what one SequenceAligner fed the same batches flags.
"""
from collections import deque

from . import _native
from .alignment import score as _score
from .alignment.aligner import AlignmentResult, _as_bytes
from .ds.sequence import Sequence


class AlignStream:
    def __init__(self, mode, score, a, b, device=0, handles=4, pipeline=2, raw=False,
                 shared=True):
        """raw=True: results are Handle.fetch_raw() records (status / score / offset / len
        lists and the two string buffers, valid until the same handle is collected again)
        instead of AlignmentResult objects — for throughput measurement (bench.py).
        pipeline: each handle's slots (>= 2 plans the DP with room for the traceback beside it,
        which the rotation puts there).  shared=False: every handle on streams of its own (the
        round-4 layout, kept for comparison)."""
        if handles < 1:
            raise ValueError("handles must be >= 1")
        self.raw = raw
        self.mode, self.score, self.a, self.b = mode, score, int(a), int(b)
        first = _native.Handle(device)
        self._hs = [first] + [_native.Handle(device, share=first if shared else None)
                              for _ in range(handles - 1)]
        for h in self._hs:
            h.set_pipeline(pipeline)
            if shared:
                h.set_async_fetch(True)
        self._next = 0
        self._inflight = deque()            # (handle index, tag, panics, pairs-or-None)
        # batches collected to free a handle whose submit then failed (prepare / execute raised):
        # handed out first by the next submit or drain, so no result is lost
        self._pending = []
        # the stream is ONE reference aligner: its scratch dims (aligner.rs:92-94, which decide
        # the reference-divergence flag, status 4) pass from handle to handle in call order
        self._buf = self._hs[0].buffer_size()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _collect(self):
        hi, tag, panics, keys = self._inflight.popleft()
        if self.raw:
            return tag, self._hs[hi].fetch_raw()
        out = self._hs[hi].fetch()
        res = []
        for p, r in enumerate(out):
            if r["status"] == 0 and panics and keys is not None and \
                    _score.pair_panics(panics, keys[p][0], keys[p][1]):
                r = dict(r, status=_native.BG_UNSCORABLE)
            res.append(AlignmentResult(r["score"], Sequence(r["aligned1"]), Sequence(r["aligned2"]),
                                       r["status"], r["end"], r["start"]))
        return tag, res

    def _slot(self):
        """The next handle of the rotation, after collecting the batch it still holds (plus any
        batches a failed submit collected earlier)."""
        ready, self._pending = self._pending, []
        hi = self._next
        if any(x[0] == hi for x in self._inflight):
            while self._inflight and self._inflight[0][0] != hi:
                ready.append(self._collect())
            ready.append(self._collect())
        self._next = (hi + 1) % len(self._hs)
        return hi, ready

    def submit(self, pairs, tag=None):
        """Queues one batch of (seq1, seq2) pairs.  Returns the batches that had to be collected
        to free a handle: a list of (tag, results), oldest first."""
        pairs = [(_as_bytes(x), _as_bytes(y)) for x, y in pairs]
        sc, panics = _score.tabulate(self.score, pairs)
        hi, ready = self._slot()
        h = self._hs[hi]
        try:
            h.set_buffer_size(*self._buf)
            h.prepare(self.mode, pairs, sc, self.a, self.b)
            self._buf = h.buffer_size()
            h.execute()
        except Exception:
            self._pending = ready           # returned by the next submit / drain
            raise
        self._inflight.append((hi, tag, panics, pairs if panics else None))
        return ready

    def submit_packed(self, buf1, off1, idx1, buf2, off2, idx2, tag=None):
        """Queues the pairs (buf1[off1[idx1[p]]:off1[idx1[p]+1]], the same in buf2) straight from
        packed residue buffers — FastaBatch.seq / .offsets — with no per-pair copy."""
        sc, panics = _score.tabulate(self.score, [(buf1, buf2)])
        hi, ready = self._slot()
        h = self._hs[hi]
        try:
            h.set_buffer_size(*self._buf)
            h.prepare_packed(self.mode, buf1, off1, idx1, buf2, off2, idx2, sc, self.a, self.b)
            self._buf = h.buffer_size()
            h.execute()
        except Exception:
            self._pending = ready
            raise
        keys = None
        if panics:
            keys = [(buf1[off1[i]:off1[i + 1]], buf2[off2[j]:off2[j + 1]]) for i, j in zip(idx1, idx2)]
        self._inflight.append((hi, tag, panics, keys))
        return ready

    def drain(self):
        """Collects every batch still in flight: a list of (tag, results), oldest first."""
        out, self._pending = self._pending, []
        while self._inflight:
            out.append(self._collect())
        return out

    def host_timing(self, reset=False):
        """Host-side ms per prepare / fetch phase summed over the rotation's handles
        (Handle.host_timing)."""
        tot = {}
        for h in self._hs:
            for k, v in h.host_timing(reset).items():
                tot[k] = max(tot.get(k, 0), v) if k == "host_threads" else tot.get(k, 0) + v
        return tot

    def close(self):
        for h in self._hs:
            h.close()
        self._hs = []
        self._inflight.clear()
        self._pending = []


def align_stream(mode, batches, score, a, b, **kw):
    """Generator over (tag, results) for an iterable of (tag, pairs) batches, in order."""
    with AlignStream(mode, score, a, b, **kw) as st:
        for tag, pairs in batches:
            yield from st.submit(pairs, tag=tag)
        yield from st.drain()
