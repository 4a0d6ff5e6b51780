"""The multi-GPU data path on the device: bg_batch_export packs a
rank's results on the GPU; the record decodes to exactly what bg_batch_fetch returns; it travels
through shard.gather_packed over RCCL (a world-size-1 "nccl" group: one GPU on this box); and a
batch LPT-sharded over several handles, exported and merged, equals the single-handle run."""
import os
import random
import socket

import pytest

from parity_util import DNA, mutate, rand_seq

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def torch_hip_first():
    """torch ships its own HIP runtime (torch/lib/libamdhip64.so); it must initialise before the
    library's (/opt/rocm) does in this process, as bench.py does, or torch sees no GPU."""
    import torch
    torch.cuda.init()
    yield


def _pairs(seed, n=61):
    rng = random.Random(seed)
    out = []
    for k in range(n):
        s1 = rand_seq(rng, rng.choice([0, 1, 63, 150, 700, 2500]), DNA)
        s2 = mutate(rng, s1, DNA, 0.15) if k % 3 else rand_seq(rng, rng.randint(0, 3000), DNA)
        out.append((s1, s2))
    return out


def _export(h):
    import torch
    from biogarden_amd import _native
    n = h.export_size()
    buf = torch.empty(max(n, 1), dtype=torch.uint8, device="cuda")
    h.export_to(buf.data_ptr(), n)
    torch.cuda.synchronize()
    return buf[:n], _native.decode_export(buf[:n].cpu().numpy().tobytes())


@pytest.mark.parametrize("mode,a,b", [("semiglobal", -1, -2), ("global", -11, -1), ("local", -11, -1)])
def test_export_record_decodes_to_fetch(mode, a, b):
    from biogarden_amd import _native
    h = _native.Handle(0)
    try:
        h.prepare(mode, _pairs(5), _native.builtin_scoring(_native.BG_BLOSUM62), a, b)
        h.execute()
        fetched = h.fetch()
        _, decoded = _export(h)
        assert decoded == fetched
    finally:
        h.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gather_over_rccl_world1():
    """shard.gather_packed over a real RCCL communicator (backend "nccl" on ROCm)."""
    import torch
    import torch.distributed as dist
    from biogarden_amd import _native, shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    h = _native.Handle(0)
    try:
        h.prepare("semiglobal", _pairs(9), _native.builtin_scoring(_native.BG_BLOSUM62), -1, -2)
        h.execute()
        fetched = h.fetch()
        local, _ = _export(h)
        got = shard.gather_packed(local, dist, dst=0)
        assert len(got) == 1
        assert _native.decode_export(got[0]) == fetched
    finally:
        h.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_lpt_sharded_handles_merge_to_single_run(world):
    """One batch LPT-sharded over `world` handles (each standing in for a rank's GPU), packed
    by bg_batch_export, decoded and merged in caller order = one handle over the whole batch."""
    from biogarden_amd import _native, shard
    sc = _native.builtin_scoring(_native.BG_BLOSUM62)
    pairs = _pairs(17 + world)
    # an empty seq1 against a long seq2 resizes the reference's scratch to 1 x 3501 (flagged
    # itself, aligner.rs:98-104); the calls after it then run on one row until a longer seq1
    # resizes again (flagged when len1 == 1): the statuses depend on the whole batch's history
    pairs[5:5] = [(b"", bytes(random.Random(3).choice(b"ACGT") for _ in range(3500)))]
    pairs[6:6] = [(b"A", b"ACGT"), (b"C", b"CCGTA")]
    h = _native.Handle(0)
    try:
        single = h.align_batch("global", pairs, sc, -11, -1)
    finally:
        h.close()
    sizes = [(len(x), len(y)) for x, y in pairs]
    shards = shard.lpt_shards(sizes, world)
    per = []
    for idx in shards:
        hr = _native.Handle(0)
        try:
            # status 4 is judged against the scratch dims one reference aligner running the whole
            # batch would hold before each call (aligner.rs:92-94): every rank replays that history
            hr.set_call_dims(shard.shard_call_dims("global", sizes, -11, -1, idx))
            hr.prepare("global", [pairs[p] for p in idx], sc, -11, -1)
            hr.execute()
            hr.synchronize()
            per.append(_export(hr)[1])
        finally:
            hr.close()
    merged = shard.merge_shards(shards, per)
    assert [r["status"] for r in single].count(4) > 0      # the flag is exercised
    assert merged == single


def test_call_dims_mismatch_is_rejected():
    from biogarden_amd import _native
    h = _native.Handle(0)
    try:
        h.set_call_dims([(1024, 1024)] * 3)
        with pytest.raises(RuntimeError):
            h.prepare("global", _pairs(1, n=2), _native.builtin_scoring(_native.BG_BLOSUM62), -11, -1)
        # a rejected prepare leaves them pending: the batch they were set for still takes them
        # (and consumes them), after which the handle runs from its own history again
        h.prepare("global", _pairs(1, n=3), _native.builtin_scoring(_native.BG_BLOSUM62), -11, -1)
        h.prepare("global", _pairs(1, n=2), _native.builtin_scoring(_native.BG_BLOSUM62), -11, -1)
    finally:
        h.close()


def _compact(h):
    import torch
    n = h.export_compact_size()
    buf = torch.empty(max(n, 1), dtype=torch.uint8, device="cuda")
    h.export_compact_to(buf.data_ptr(), n)
    torch.cuda.synchronize()
    return buf[:n].cpu().numpy().tobytes()


@pytest.mark.parametrize("mode,a,b", [("semiglobal", -1, -2), ("semiglobal", -11, -1), ("global", -11, -1),
                                      ("local", -11, -1), ("fitting", -1, -1), ("overlap", -2, -2)])
def test_compact_export_expands_to_fetch(mode, a, b):
    """bg_batch_export_compact (headers + 2-bit edit scripts of the alignment cores, the gather
    payload) expanded on the host with the input sequences = bg_batch_fetch, pair for pair:
    semiglobal prefixes / tails, empty and unscorable pairs (status 3), divergence flags."""
    from biogarden_amd import _native
    pairs = _pairs(23 + len(mode) + a)
    pairs += [(b"ACGTNNACGT", b"ACGT"), (b"", b"ACG"), (b"A", b""), (b"ACGTZACGT", b"ACGT")]
    pairs += [(b"ACGT" * 40, b"AC!GT")]                     # '!' is outside score.rs's table: status 3
    h = _native.Handle(0)
    try:
        h.prepare(mode, pairs, _native.builtin_scoring(_native.BG_BLOSUM62), a, b)
        h.execute()
        fetched = h.fetch()
        rec = _compact(h)
    finally:
        h.close()
    assert _native.expand_compact(rec, pairs) == fetched
    assert any(r["status"] == 3 for r in fetched)
    full = 8 + 40 * len(pairs) + 2 * sum(len(x) + len(y) for x, y in pairs)
    assert len(rec) < full / 4, (len(rec), full)


def test_compact_export_with_gap_byte_residues():
    """A closure over raw bytes where '-' itself is a residue (the reference's scorer is any
    &dyn Fn(&u8, &u8) -> i32): the edit script, not the strings, carries the gaps, so the
    expansion is still exact."""
    from biogarden_amd import _native
    from biogarden_amd.alignment import score
    alpha = b"-ACGT"
    rng = random.Random(8)
    pairs = []
    for n1, n2 in ((300, 280), (64, 65), (1000, 700), (5, 0)):
        s1 = rand_seq(rng, n1, alpha)
        pairs.append((s1, mutate(rng, s1, alpha, 0.2)[:n2]))
    sc, _ = score.tabulate(lambda x, y: 5 if x == y else -4, pairs)
    h = _native.Handle(0)
    try:
        h.prepare("global", pairs, sc, -6, -1)
        h.execute()
        fetched = h.fetch()
        rec = _compact(h)
    finally:
        h.close()
    assert _native.expand_compact(rec, pairs) == fetched
    assert any(b"-" in x for x, _ in pairs)


def test_compact_gather_over_rccl_world1():
    import torch
    import torch.distributed as dist
    from biogarden_amd import _native, shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    pairs = _pairs(31)
    h = _native.Handle(0)
    try:
        h.prepare("semiglobal", pairs, _native.builtin_scoring(_native.BG_BLOSUM62), -1, -2)
        h.execute()
        fetched = h.fetch()
        n = h.export_compact_size()
        buf = torch.empty(max(n, 1), dtype=torch.uint8, device="cuda")
        h.export_compact_to(buf.data_ptr(), n)
        got = shard.gather_packed(buf[:n], dist, dst=0)
        assert _native.expand_compact(got[0], pairs) == fetched
    finally:
        h.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,a,b", [("semiglobal", -1, -2), ("local", -11, -1)])
def test_compact_export_async_pipelined(mode, a, b):
    """bg_batch_export_compact_async (the strong bench step): every execute's record exported
    without a host wait into a buffer of its own, six executes pipelined over three arena slots
    (each slot's next execute waits for its export), torch's stream ordered after each record;
    every record equals the synchronous export of the same batch, bytes for bytes, and fits the
    bound."""
    import struct

    import torch
    from biogarden_amd import _native
    pairs = _pairs(41 + len(mode))
    h = _native.Handle(0)
    try:
        h.set_pipeline(3)
        h.prepare(mode, pairs, _native.builtin_scoring(_native.BG_BLOSUM62), a, b)
        cap = h.export_compact_bound()
        bufs = [torch.full((cap,), 0xAB, dtype=torch.uint8, device="cuda") for _ in range(6)]
        stream = torch.cuda.current_stream()
        for buf in bufs:
            h.execute()
            h.export_compact_async(buf.data_ptr(), cap, stream.cuda_stream)
        copies = [buf.cpu() for buf in bufs]          # on torch's stream: after each record
        ref = _compact(h)
        fetched = h.fetch()
    finally:
        h.close()
    assert len(ref) <= cap
    for c in copies:
        raw = c.numpy().tobytes()
        _, n, ops, _ = struct.unpack_from("<4Q", raw, 0)
        assert 32 + 48 * n + ops == len(ref)
        assert raw[:len(ref)] == ref
    assert _native.expand_compact(ref, pairs) == fetched
