"""Streaming ingest on the GPU (biogarden_amd.stream): reads and refs
written as FASTA, read back in batches by the native BatchReader, queued through AlignStream's
handle rotation straight from the packed batch buffers — every result (status, score, both
aligned strings) is compared with the CPU oracle: the exact-size answer, and the status a
reference-faithful aligner fed the same pairs in submission order would earn (the stream stands
for ONE SequenceAligner, aligner.rs:92-94)."""
import random

import pytest

from parity_util import DNA, check_results, mutate, rand_seq

pytestmark = pytest.mark.gpu


def _write_fasta(path, recs):
    with open(path, "w") as f:
        for i, s in enumerate(recs):
            f.write(">r%d some desc\n" % i)
            for k in range(0, len(s), 60):
                f.write(s[k:k + 60].decode() + "\n")


@pytest.mark.parametrize("handles", [1, 2, 4])
def test_fasta_reads_vs_refs_streamed(tmp_path, handles, oracle):
    from biogarden_amd.alignment import score
    from biogarden_amd.alignment.aligner import SequenceAligner
    from biogarden_amd.io import fasta
    from biogarden_amd.stream import AlignStream
    rng = random.Random(handles)
    refs = [rand_seq(rng, 3000, DNA) for _ in range(3)]
    reads, which = [], []
    for k in range(300):
        r = k % 3
        o = rng.randint(0, 2800)
        reads.append(mutate(rng, refs[r][o:o + rng.randint(50, 200)], DNA, 0.04))
        which.append(r)
    _write_fasta(tmp_path / "refs.fa", refs)
    _write_fasta(tmp_path / "reads.fa", reads)
    rb = next(iter(fasta.BatchReader(str(tmp_path / "refs.fa"))))
    got = []
    base = 0
    with AlignStream("semiglobal", score.blosum62, -1, -2, handles=handles) as st:
        for b in fasta.BatchReader(str(tmp_path / "reads.fa"), max_records=70):
            idx = list(range(len(b)))
            got += st.submit_packed(b.seq, b.offsets, idx, rb.seq, rb.offsets,
                                    [which[base + i] for i in idx], tag=base)
            base += len(b)
        got += st.drain()
    assert [t for t, _ in got] == sorted(t for t, _ in got)
    flat = [r for _, rs in got for r in rs]
    assert len(flat) == 300
    pairs = [(reads[i], refs[which[i]]) for i in range(len(reads))]
    check_results(oracle, "semiglobal", pairs, flat, "blosum62", -1, -2, dims=(1024, 1024))
    # and the same as one aligner's batch (end cells included)
    al = SequenceAligner(0)
    try:
        want = al.align_batch("semiglobal", pairs, score.blosum62, -1, -2)
    finally:
        al.close()
    assert [r.end for r in flat] == [r.end for r in want]


def test_align_stream_generator_mixed_batches(oracle):
    from biogarden_amd.alignment import score
    from biogarden_amd.stream import align_stream
    rng = random.Random(7)
    batches = []
    for t in range(7):
        pairs = []
        for _ in range(rng.randint(0, 40)):
            s1 = rand_seq(rng, rng.randint(0, 900), DNA)
            pairs.append((s1, mutate(rng, s1, DNA, 0.1)))
        batches.append((t, pairs))
    out = list(align_stream("global", batches, score.blosum62, -11, -1, handles=3))
    assert [t for t, _ in out] == list(range(7))
    ref = oracle.Aligner(dims=(1024, 1024))      # one reference aligner across every batch
    for (t, pairs), (_, res) in zip(batches, out):
        assert len(res) == len(pairs)
        check_results(oracle, "global", pairs, res, "blosum62", -11, -1, ref=ref)


def test_failed_submit_keeps_collected_results(oracle):
    """A submit that has to collect a finished batch to free its handle and then fails in
    prepare hands the collected batch out with the next submit / drain: nothing is lost."""
    from biogarden_amd.alignment import score
    from biogarden_amd.stream import AlignStream
    rng = random.Random(11)
    batches = [[(rand_seq(rng, 200, DNA), rand_seq(rng, 180, DNA)) for _ in range(5)] for _ in range(4)]
    seen = []
    with AlignStream("global", score.blosum62, -11, -1, handles=2) as st:
        seen += st.submit(batches[0], tag=0)
        seen += st.submit(batches[1], tag=1)            # the rotation is full
        st.mode = 99                                    # an unknown mode: prepare fails (BG_E_ARG)
        with pytest.raises(RuntimeError):
            st.submit(batches[2], tag=2)                # collected batch 0 first
        st.mode = "global"
        seen += st.submit(batches[3], tag=3)
        seen += st.drain()
    assert [t for t, _ in seen] == [0, 1, 3]
    for t, res in seen:
        check_results(oracle, "global", batches[t], res, "blosum62", -11, -1)


def test_shared_stream_handles_hold_independent_batches(oracle):
    """Handles sharing one stream set (bg_aligner_new_shared) hold different batches in flight at
    once: every fetch waits for its own handle's work only, in any order; an asynchronous fetch
    (bg_set_async_fetch, the download queued behind the traceback) returns what a plain fetch
    returns, also after several executes of one batch."""
    from biogarden_amd import _native
    rng = random.Random(99)
    jobs = [("global", -11, -1), ("semiglobal", -1, -2), ("local", -11, -1), ("overlap", -2, -3)]
    batches = []
    for _ in jobs:
        pairs = []
        for _ in range(rng.randint(20, 60)):
            s1 = rand_seq(rng, rng.randint(0, 2500), DNA)
            pairs.append((s1, mutate(rng, s1, DNA, 0.12)[: rng.randint(0, 2600)]))
        batches.append(pairs)
    sc = _native.builtin_scoring(_native.BG_BLOSUM62)
    first = _native.Handle(0)
    hs = [first] + [_native.Handle(share=first) for _ in jobs[1:]]
    try:
        for k, h in enumerate(hs):
            h.set_pipeline(1 + k % 3)
            if k % 2:
                h.set_async_fetch(True)
        for h, (mode, a, b), pairs in zip(hs, jobs, batches):
            h.prepare(mode, pairs, sc, a, b)
            h.execute()
        for k in (2, 0, 3, 1):
            mode, a, b = jobs[k]
            got = hs[k].fetch()
            check_results(oracle, mode, batches[k], [_res(r) for r in got], "blosum62", a, b,
                          dims=(1024, 1024))
        # several executes of one batch in flight beside another handle's, then one fetch
        hs[1].execute()
        hs[3].execute()
        hs[1].execute()
        hs[1].execute()
        again = hs[1].fetch()
        first_run = hs[3].fetch()
        mode, a, b = jobs[1]
        check_results(oracle, mode, batches[1], [_res(r) for r in again], "blosum62", a, b,
                      dims=(1024, 1024))
        mode, a, b = jobs[3]
        check_results(oracle, mode, batches[3], [_res(r) for r in first_run], "blosum62", a, b,
                      dims=(1024, 1024))
    finally:
        for h in reversed(hs):
            h.close()


def _res(r):
    from biogarden_amd.alignment.aligner import AlignmentResult
    from biogarden_amd.ds.sequence import Sequence
    return AlignmentResult(r["score"], Sequence(r["aligned1"]), Sequence(r["aligned2"]), r["status"],
                           r["end"], r["start"])


@pytest.mark.parametrize("shared", [True, False])
def test_stream_shared_and_unshared_agree(oracle, shared):
    """The rotation on one shared stream set with asynchronous downloads (the default) and on
    streams of its own per handle give the same results, batch for batch."""
    from biogarden_amd.alignment import score
    from biogarden_amd.stream import AlignStream
    rng = random.Random(5)
    batches = []
    for t in range(6):
        pairs = [(rand_seq(rng, rng.randint(100, 3000), DNA), rand_seq(rng, rng.randint(100, 3000), DNA))
                 for _ in range(rng.randint(1, 30))]
        batches.append(pairs)
    out = []
    with AlignStream("semiglobal", score.blosum62, -1, -2, handles=3, shared=shared) as st:
        for t, pairs in enumerate(batches):
            out += st.submit(pairs, tag=t)
        out += st.drain()
    assert [t for t, _ in out] == list(range(6))
    ref = oracle.Aligner(dims=(1024, 1024))
    for (t, res), pairs in zip(out, batches):
        check_results(oracle, "semiglobal", pairs, res, "blosum62", -1, -2, ref=ref)
