"""Multi-rank plumbing on CPU (gloo, world size 2): shard -> per-rank packed results ->
variable-size gather -> decode -> merge, as bench.py / biogarden_amd.shard do over RCCL."""
import os
import random
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from biogarden_amd import _native, shard  # noqa: E402


def _fake_results(pairs, seed):
    rng = random.Random(seed)
    out = []
    for s1, s2 in pairs:
        L = len(s1) + len(s2) - rng.randint(0, min(len(s1), len(s2)))
        a1 = bytes(rng.choice(b"ACGT-") for _ in range(L))
        a2 = bytes(rng.choice(b"ACGT-") for _ in range(L))
        out.append({"status": rng.choice([0, 0, 0, 4]), "score": rng.randint(-50, 500),
                    "aligned1": a1, "aligned2": a2, "end": (len(s1), len(s2)),
                    "start": (rng.randint(0, 3), rng.randint(0, 3))})
    return out


def _pairs(n, seed):
    rng = random.Random(seed)
    return [(bytes(rng.choice(b"ACGT") for _ in range(rng.randint(0, 40))),
             bytes(rng.choice(b"ACGT") for _ in range(rng.randint(0, 40)))) for _ in range(n)]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pairs = _pairs(23, 7)
        shards = shard.lpt_shards([(len(a), len(b)) for a, b in pairs], world)
        mine = [pairs[p] for p in shards[rank]]
        res = _fake_results(mine, 100 + rank)
        local = torch.frombuffer(bytearray(shard.encode_export(res)), dtype=torch.uint8)
        got = shard.gather_packed(local, dist, dst=0)
        if rank == 0:
            decoded = [_native.decode_export(b) for b in got]
            expect = [_fake_results([pairs[p] for p in shards[r]], 100 + r) for r in range(world)]
            merged = shard.merge_shards(shards, decoded)
            q.put(("ok", decoded == expect, len(merged), all(m is not None for m in merged)))
    except Exception as e:  # surface worker failures to the test
        q.put(("err", repr(e)))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _oracle_results(pairs, mode, a, b):
    """What a rank's bg_batch_fetch returns for its shard, computed by the CPU oracle (the GPU
    path is bit-exact with it, tests/test_gpu_*.py): status, score and both aligned strings."""
    from oracle import refcpu
    out = []
    for s1, s2 in pairs:
        st, sc, o1, o2 = refcpu.align(mode, s1, s2, "blosum62", a, b, exact=True)
        out.append({"status": st, "score": sc, "aligned1": o1, "aligned2": o2,
                    "end": (len(s1), len(s2)), "start": (0, 0)})
    return out


def _real_pairs(n, seed):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        s1 = bytes(rng.choice(b"ACGT") for _ in range(rng.randint(0, 300)))
        s2 = bytearray(s1[rng.randint(0, len(s1)):] if s1 else b"")
        for k in range(len(s2)):
            if rng.random() < 0.1:
                s2[k] = rng.choice(b"ACGT")
        s2 = bytes(s2) + bytes(rng.choice(b"ACGT") for _ in range(rng.randint(0, 60)))
        out.append((s1, s2))
    return out


def _sharded_worker(rank, world, port, q, mode, a, b):
    """One rank of a sharded batch: LPT shard -> align its pairs -> pack them in
    bg_batch_export's record layout -> variable-size gather to rank 0 -> decode + merge in
    the caller's pair order."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pairs = _real_pairs(37, 11)
        shards = shard.lpt_shards([(len(x), len(y)) for x, y in pairs], world)
        mine = _oracle_results([pairs[p] for p in shards[rank]], mode, a, b)
        local = torch.frombuffer(bytearray(shard.encode_export(mine)), dtype=torch.uint8)
        got = shard.gather_packed(local, dist, dst=0)
        if rank == 0:
            merged = shard.merge_shards(shards, [_native.decode_export(x) for x in got])
            single = _oracle_results(pairs, mode, a, b)
            q.put(("ok", merged == single, len(merged), [len(s) for s in shards]))
        else:
            q.put(("rank", rank, got is None))
    except Exception as e:  # surface worker failures to the test
        q.put(("err", repr(e)))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _faithful_results(pairs, mode, a, b, dims):
    """What a rank's fetch returns for its shard when every call starts from the scratch dims a
    single reference aligner would hold (shard.call_dims): the reference-faithful oracle from
    those dims (status 4 where it panics or its answer differs from the exact-size one)."""
    from oracle import refcpu
    out = []
    for (s1, s2), d in zip(pairs, dims):
        st, sc, o1, o2 = refcpu.align(mode, s1, s2, "blosum62", a, b, exact=True)
        fst, fsc, f1, f2 = refcpu.Aligner(dims=d).align(mode, s1, s2, "blosum62", a, b)
        if st == 0 and not (fst == 0 and (fsc, f1, f2) == (sc, o1, o2)):
            st = 4
        out.append({"status": st, "score": sc, "aligned1": o1, "aligned2": o2,
                    "end": (len(s1), len(s2)), "start": (0, 0)})
    return out


def _c4_like_pairs():
    """C4's shape (150 bp reads with 2 % substitutions against 10 kbp refs, seq1 = read) plus
    calls whose statuses depend on the batch's history: after a 1100 x 1100 call resized the
    scratch to 1101 x 1101, a 1101-long seq1 and a 1101-long seq2 (equal to the rows / columns:
    the reference panics, aligner.rs:92-94) and a 1099 x 700 one (it does not)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from tools import workloads
    pairs = workloads.c4_pairs(nrefs=2, reads_per_ref=6)
    rng = random.Random(5)
    seq = lambda n: bytes(rng.choice(b"ACGT") for _ in range(n))  # noqa: E731
    pairs[3:3] = [(seq(1100), seq(1100)), (seq(1101), seq(700)), (seq(150), seq(1101)),
                  (seq(1099), seq(700))]
    return pairs


def _c4_sharded_worker(rank, world, port, q):
    """A C4-shaped batch through the multi-rank path with the whole batch's call history."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        mode, a, b = "semiglobal", -1, -2
        pairs = _c4_like_pairs()
        sizes = [(len(x), len(y)) for x, y in pairs]
        shards = shard.lpt_shards(sizes, world)
        dims = shard.shard_call_dims(mode, sizes, a, b, shards[rank])
        mine = _faithful_results([pairs[p] for p in shards[rank]], mode, a, b, dims)
        local = torch.frombuffer(bytearray(shard.encode_export(mine)), dtype=torch.uint8)
        got = shard.gather_packed(local, dist, dst=0)
        if rank == 0:
            merged = shard.merge_shards(shards, [_native.decode_export(x) for x in got])
            single = _faithful_results(pairs, mode, a, b, shard.call_dims(mode, sizes, a, b))
            # the sequential reference aligner over the whole batch, for the statuses
            from oracle import refcpu
            al = refcpu.Aligner(exact=False)
            seq_st = []
            for s1, s2 in pairs:
                fst = al.align(mode, s1, s2, "blosum62", a, b)
                seq_st.append(fst)
            q.put(("ok", merged == single, [r["status"] for r in merged],
                   [(f[0], f[1:]) for f in seq_st], [r["score"] for r in single],
                   [(r["aligned1"], r["aligned2"]) for r in single]))
        else:
            q.put(("rank", rank, got is None))
    except Exception as e:  # surface worker failures to the test
        q.put(("err", repr(e)))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_c4_shaped_shards_equal_one_reference_aligner(world):
    """C4-shaped pairs sharded over gloo ranks, each rank starting its calls from the whole
    batch's scratch history: merged statuses, scores and strings equal ONE reference aligner
    running the batch in order (status 4 exactly where that aligner panics or answers from
    stale scratch)."""
    msgs, procs = _run_world(_c4_sharded_worker, world, timeout=300)
    ok = [m for m in msgs if m[0] == "ok"]
    assert len(ok) == 1, msgs
    _, same, statuses, seq, scores, strings = ok[0]
    assert same
    for st, (fst, (fsc, f1, f2)), sc, (o1, o2) in zip(statuses, seq, scores, strings):
        if fst == 0 and (fsc, f1, f2) == (sc, o1, o2):
            assert st == 0
        else:
            assert st == 4
    assert statuses[4] == 4 and statuses[5] == 4 and statuses[6] == 0, statuses
    assert all(p.exitcode == 0 for p in procs)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_batch_equals_single_rank(world):
    """The multi-rank data path on CPU ranks: the merged gather of every rank's packed shard
    equals a single-rank run of the same pairs, pair for pair (status, score, both strings)."""
    msgs, procs = _run_world(_sharded_worker, world, ("semiglobal", -11, -1))
    ok = [m for m in msgs if m[0] == "ok"]
    assert len(ok) == 1, msgs
    assert ok[0][1] and ok[0][2] == 37 and min(ok[0][3]) > 0, ok
    assert all(m[0] in ("ok", "rank") for m in msgs), msgs
    assert all(p.exitcode == 0 for p in procs)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_world(target, world, extra=(), nmsgs=None, timeout=180):
    """Spawns `world` gloo ranks of target(rank, world, port, q, *extra) and returns (messages,
    processes).  A port taken between _free_port and the store's bind (another process on the
    machine) fails rank 0's init with EADDRINUSE: that try is torn down and run again on a fresh
    port, at most three times."""
    ctx = mp.get_context("spawn")
    nmsgs = world if nmsgs is None else nmsgs
    for attempt in range(3):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=target, args=(r, world, port, q) + tuple(extra)) for r in range(world)]
        for p in procs:
            p.start()
        msgs = []
        while len(msgs) < nmsgs:
            msgs.append(q.get(timeout=timeout))
            if msgs[-1][0] == "err" and "EADDRINUSE" in msgs[-1][1] and attempt < 2:
                break
        else:
            for p in procs:
                p.join(timeout=120)
            return msgs, procs
        for p in procs:
            p.kill()
            p.join(timeout=30)
    raise AssertionError("unreachable")


def test_lpt_shards_balance_and_cover():
    sizes = [(random.Random(i).randint(0, 1000), random.Random(i + 99).randint(0, 1000)) for i in range(101)]
    sh = shard.lpt_shards(sizes, 4)
    assert sorted(p for s in sh for p in s) == list(range(101))
    loads = [sum(sizes[p][0] * sizes[p][1] for p in s) for s in sh]
    assert max(loads) - min(loads) <= max(a * b for a, b in sizes)


def test_encode_decode_roundtrip():
    res = _fake_results(_pairs(9, 3), 5)
    assert _native.decode_export(shard.encode_export(res)) == res
    assert _native.decode_export(shard.encode_export([])) == []


def test_gather_two_ranks_gloo():
    (msg,), procs = _run_world(_worker, 2, nmsgs=1, timeout=120)
    assert msg[0] == "ok", msg
    assert msg[1] and msg[2] == 23 and msg[3]
    assert all(p.exitcode == 0 for p in procs)


@pytest.mark.parametrize("mode,a,b", [("global", -11, -1), ("local", -11, -1), ("fitting", -1, -1),
                                      ("overlap", -2, -2), ("semiglobal", -1, -2),
                                      ("global", 1, -1)])
def test_call_dims_follow_the_reference_aligner(mode, a, b):
    """shard.call_dims (the per-pair scratch dims every rank replays over the whole batch) equals
    the dims a reference-faithful SequenceAligner (oracle/refcpu.c, aligner.rs:44-55, 92-94,
    594-602) holds before each call, through argument errors, fitting's size error, equal-size
    and larger pairs."""
    from oracle import refcpu
    rng = random.Random(hash((mode, a, b)) & 0xFFFF)
    lens = [0, 1, 2, 7, 40, 1023, 1024, 1025, 1100]
    pairs = [(bytes(rng.choice(b"ACGT") for _ in range(rng.choice(lens))),
              bytes(rng.choice(b"ACGT") for _ in range(rng.choice(lens)))) for _ in range(24)]
    al = refcpu.Aligner(exact=False)
    want = []
    for s1, s2 in pairs:
        want.append(al.buffer_size())
        al.align(mode, s1, s2, "blosum62", a, b)
    got = shard.call_dims(mode, [(len(x), len(y)) for x, y in pairs], a, b)
    assert got == want
    idx = [3, 0, 17, 9]
    assert shard.shard_call_dims(mode, [(len(x), len(y)) for x, y in pairs], a, b, idx) == \
        [want[p] for p in idx]


def test_group_plan_matches_rank_sharding():
    """bg_group_plan (the C ABI's multi-device split, host-only) assigns every pair to the shard
    shard.lpt_shards gives it: the single-process group and the one-process-per-GPU ranks split a
    batch the same way."""
    import random
    from biogarden_amd import _native, shard
    rng = random.Random(8)
    for _ in range(40):
        n = rng.randint(0, 400)
        k = rng.randint(1, 9)
        sizes = [(rng.choice([0, 1, 150, 1000, rng.randint(0, 9000)]),
                  rng.choice([0, 10, 10000, rng.randint(0, 9000)])) for _ in range(n)]
        got = _native.group_plan(sizes, k)
        want = shard.lpt_shards(sizes, k)
        assert [[p for p in range(n) if got[p] == r] for r in range(k)] == want
