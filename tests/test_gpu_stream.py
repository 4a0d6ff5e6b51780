"""Streaming ingest on the GPU (biogarden_amd.stream): reads and refs
written as FASTA, read back in batches by the native BatchReader, queued through AlignStream's
handle rotation straight from the packed batch buffers — every result (status, score, both
aligned strings) equals one SequenceAligner.align_batch over the same pairs, in submission order."""
import random

import pytest

from parity_util import DNA, mutate, rand_seq

pytestmark = pytest.mark.gpu


def _write_fasta(path, recs):
    with open(path, "w") as f:
        for i, s in enumerate(recs):
            f.write(">r%d some desc\n" % i)
            for k in range(0, len(s), 60):
                f.write(s[k:k + 60].decode() + "\n")


@pytest.mark.parametrize("handles", [1, 2, 4])
def test_fasta_reads_vs_refs_streamed(tmp_path, handles):
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
    al = SequenceAligner(0)
    try:
        want = al.align_batch("semiglobal", [(reads[i], refs[which[i]]) for i in range(len(reads))],
                              score.blosum62, -1, -2)
    finally:
        al.close()
    key = lambda r: (r.status, r[0], bytes(r[1].chain), bytes(r[2].chain), r.end)  # noqa: E731
    assert len(flat) == len(want) == 300
    assert [key(r) for r in flat] == [key(r) for r in want]


def test_align_stream_generator_mixed_batches():
    from biogarden_amd.alignment import score
    from biogarden_amd.alignment.aligner import SequenceAligner
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
    al = SequenceAligner(0)
    try:
        for (t, pairs), (_, res) in zip(batches, out):
            want = al.align_batch("global", pairs, score.blosum62, -11, -1) if pairs else []
            assert [(r[0], bytes(r[1].chain), bytes(r[2].chain)) for r in res] == \
                   [(r[0], bytes(r[1].chain), bytes(r[2].chain)) for r in want]
    finally:
        al.close()
