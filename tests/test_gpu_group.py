"""Several GPUs from one process through the C ABI (bg_group): a batch split over
members by cells, every shard aligned on its member's device and packed into a compact record,
the records gathered to the first member's device (RCCL send / recv; a device copy on the root
device) and expanded on the host.  The box has one GPU, so the members are virtual shards on
device 0 (they share its streams); BG_GROUP_RCCL_SELF=1 sends the root's own shards through RCCL
too (send / receive to self over a one-rank communicator), which is the path other devices take.
Every case must equal one aligner running the whole batch, byte for byte and status for status
(reference caller: tests/integration.rs:234-312, one SequenceAligner over many calls)."""
import random

import pytest

from parity_util import DNA, mutate, rand_seq

pytestmark = pytest.mark.gpu


def _single(mode, batches, a, b):
    from biogarden_amd import _native
    sc = _native.builtin_scoring(_native.BG_BLOSUM62)
    h = _native.Handle(0)
    try:
        out = []
        for pairs in batches:          # one aligner fed the batches in order (its scratch history)
            out.append(h.align_batch(mode, pairs, sc, a, b))
        return out, h.buffer_size()
    finally:
        h.close()


def _group(members, mode, batches, a, b):
    from biogarden_amd import _native
    sc = _native.builtin_scoring(_native.BG_BLOSUM62)
    g = _native.Group(members)
    try:
        out = [g.align_batch(mode, pairs, sc, a, b) for pairs in batches]
        return out, g.buffer_size(), g.timing()
    finally:
        g.close()


@pytest.mark.parametrize("rccl_self", ["0", "1"])
@pytest.mark.parametrize("members", [[0], [0, 0, 0]])
def test_group_C4_slice_equals_one_aligner(monkeypatch, rccl_self, members):
    from tools import workloads as w
    monkeypatch.setenv("BG_GROUP_RCCL_SELF", rccl_self)
    pairs = w.c4_pairs(nrefs=8, reads_per_ref=128)
    want, _ = _single("semiglobal", [pairs], -1, -2)
    got, _, tm = _group(members, "semiglobal", [pairs], -1, -2)
    assert got == want
    assert tm["calls"] == 1 and tm["gather"] > 0


def test_group_C5_share_equals_one_aligner(monkeypatch):
    from tools import workloads as w
    monkeypatch.setenv("BG_GROUP_RCCL_SELF", "1")
    pairs = w.c5_pairs(rank=0, world=8)
    want, _ = _single("global", [pairs], -11, -1)
    got, _, _ = _group([0, 0, 0, 0], "global", [pairs], -11, -1)
    assert got == want


@pytest.mark.parametrize("mode,a,b", [("global", -11, -1), ("local", -11, -1), ("semiglobal", -1, -2),
                                      ("fitting", -1, -1), ("overlap", -2, -3)])
def test_group_scratch_history_across_batches(mode, a, b):
    """Status 4 depends on the reference aligner's scratch dims after every earlier call: the
    group stands for one aligner across its batches, as the single handle does."""
    rng = random.Random(len(mode) * 7 - a)
    batches = []
    for t in range(3):
        pairs = []
        for k in range(rng.randint(5, 40)):
            s1 = rand_seq(rng, rng.choice([0, 1, 64, 150, 700, 1023, 1024, 1500, 2600]), DNA)
            s2 = mutate(rng, s1, DNA, 0.1) if k % 2 else rand_seq(rng, rng.randint(0, 2000), DNA)
            pairs.append((s1, s2))
        batches.append(pairs)
    want, dims = _single(mode, batches, a, b)
    got, gdims, _ = _group([0, 0], mode, batches, a, b)
    assert gdims == dims
    assert got == want


def test_group_more_members_than_pairs():
    rng = random.Random(3)
    pairs = [(rand_seq(rng, 300, DNA), rand_seq(rng, 280, DNA)), (b"", b"ACGT")]
    want, _ = _single("global", [pairs], -11, -1)
    got, _, _ = _group([0, 0, 0, 0, 0], "global", [pairs], -11, -1)
    assert got == want


def _decode(pairs, res, o1, o2):
    b1, b2 = bytes(o1), bytes(o2)
    out = []
    for p in range(len(pairs)):
        r = res[p]
        lo, hi = r.offset, r.offset + r.len
        out.append({"status": r.status, "score": r.score, "aligned1": b1[lo:hi], "aligned2": b2[lo:hi],
                    "end": (r.end_i, r.end_j), "start": (r.start1, r.start2)})
    return out


@pytest.mark.parametrize("rccl_self", ["0", "1"])
@pytest.mark.parametrize("mode,a,b", [("semiglobal", -1, -2), ("local", -11, -1)])
def test_group_pipelined_submit_collect(monkeypatch, rccl_self, mode, a, b):
    """bg_group_submit / bg_group_collect with three batches in flight: the same results and scratch
    history as one aligner fed the batches in order; a fourth submit and an empty collect refuse."""
    from biogarden_amd import _native
    monkeypatch.setenv("BG_GROUP_RCCL_SELF", rccl_self)
    rng = random.Random(41 + len(mode))
    batches = []
    for t in range(6):
        pairs = []
        for k in range(rng.randint(3, 30)):
            s1 = rand_seq(rng, rng.choice([0, 1, 150, 700, 1023, 1024, 1500, 2600]), DNA)
            s2 = mutate(rng, s1, DNA, 0.1) if k % 2 else rand_seq(rng, rng.randint(0, 2000), DNA)
            pairs.append((s1, s2))
        batches.append(pairs)
    want, dims = _single(mode, batches, a, b)
    sc = _native.builtin_scoring(_native.BG_BLOSUM62)
    g = _native.Group([0, 0])
    try:
        got, tickets = [], []
        for pairs in batches:
            if len(tickets) == 3:
                t = tickets.pop(0)
                got.append(_decode(t[6], *g.collect(t)))
            tickets.append(g.submit(mode, pairs, sc, a, b))
            assert g.pending() == len(tickets)
        with pytest.raises(RuntimeError):
            g.submit(mode, batches[0], sc, a, b)        # a fourth batch in flight
        with pytest.raises(RuntimeError):
            g.align_batch(mode, batches[0], sc, a, b)   # needs none pending
        while tickets:
            t = tickets.pop(0)
            got.append(_decode(t[6], *g.collect(t)))
        assert g.pending() == 0
        with pytest.raises(RuntimeError):
            g.collect((None, None, None, None, 0, 0, []))
        assert g.buffer_size() == dims
    finally:
        g.close()
    assert got == want
