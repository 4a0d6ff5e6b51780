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
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
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
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


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
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    msg = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
    assert msg[0] == "ok", msg
    assert msg[1] and msg[2] == 23 and msg[3]
    assert all(p.exitcode == 0 for p in procs)
