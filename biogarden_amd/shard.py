"""Multi-GPU plumbing for batches of independent pairs.

One process per GPU.  A batch is split over ranks by cells (largest-first greedy, like the
in-GPU pair plan); every rank runs its shard through its own `bg_aligner`, packs the results
on the device — `bg_batch_export_compact`: headers plus the alignment cores as 2-bit edit
scripts, 10-250x smaller than the strings — and rank 0 collects the records with one
variable-size gather (RCCL send/recv over xGMI with backend "nccl", gloo on CPU) and expands
them into aligned strings on the host (`_native.expand_compact`, which has the input sequences).  No collective is on
the data path: the pairs' answers share nothing (reference: one `SequenceAligner` call per
pair, src/alignment/aligner.rs:84-435).

The one thing the reference carries from call to call is its aligner's scratch dims
(aligner.rs:92-94, 594-602), which decide the reference-divergence flag (status 4).  Every rank
replays that history over the WHOLE batch in caller order (`call_dims`, a host prefix scan) and
hands its shard the dims each of its pairs starts from (`Handle.set_call_dims`), so the merged
statuses equal one aligner's run of the batch exactly.
"""
import struct

from . import _native

_NONPOS = ("global", "local", "fitting")


def call_dims(mode, sizes, a, b, start=(1024, 1024)):
    """Scratch dims each call of a batch starts from, in caller order: one reference
    SequenceAligner (1024 x 1024 when new, aligner.rs:44-55) running every pair.  A call resizes
    to (n1 + 1, n2 + 1) when n1 > rows or n2 > cols (:92-94, 594-602); the argument errors
    (InvalidArgumentRange :87-89 / 153-155 / 219-221, fitting's InvalidInputSize :223-225) return
    before that.  sizes: list of (n1, n2).  Returns a list of (rows, cols)."""
    rows, cols = start
    out = []
    bad_args = mode in _NONPOS and (a > 0 or b > 0)
    for n1, n2 in sizes:
        out.append((rows, cols))
        if bad_args or (mode == "fitting" and n1 < n2):
            continue
        if n1 > rows or n2 > cols:
            rows, cols = n1 + 1, n2 + 1
    return out


def shard_call_dims(mode, sizes, a, b, shard_idx, start=(1024, 1024)):
    """call_dims of the whole batch, restricted to one shard's pairs (in the shard's order)."""
    d = call_dims(mode, sizes, a, b, start)
    return [d[p] for p in shard_idx]


def lpt_shards(sizes, world):
    """Split pair indices over `world` ranks, balancing sum(n1 * n2): largest first, each to the
    least-loaded rank.  sizes: list of (n1, n2).  Returns `world` index lists (ascending)."""
    load = [0] * world
    shards = [[] for _ in range(world)]
    for p in sorted(range(len(sizes)), key=lambda q: (-(sizes[q][0] * sizes[q][1]), q)):
        r = min(range(world), key=lambda x: (load[x], x))
        shards[r].append(p)
        load[r] += sizes[p][0] * sizes[p][1]
    return [sorted(s) for s in shards]


def merge_shards(shards, per_rank_results):
    """Results gathered from every rank (each in its shard's order) -> one list in the
    original pair order."""
    n = sum(len(s) for s in shards)
    out = [None] * n
    for idx, res in zip(shards, per_rank_results):
        assert len(idx) == len(res)
        for p, r in zip(idx, res):
            out[p] = r
    return out


def encode_export(results):
    """Host-side encoder of the bg_batch_export record (the device kernel's format:
    [u64 n][bg_pair_result x n][aligned1 bytes][aligned2 bytes]); for tests and CPU ranks."""
    rs = []
    blob1 = bytearray()
    blob2 = bytearray()
    for r in results:
        off = len(blob1)
        a1, a2 = bytes(r["aligned1"]), bytes(r["aligned2"])
        assert len(a1) == len(a2)
        rec = _native.BgPairResult(r["status"], r["score"], off, len(a1), r["end"][0], r["end"][1],
                                   r["start"][0], r["start"][1], 0)
        rs.append(bytes(rec))
        blob1 += a1
        blob2 += a2
    return struct.pack("<Q", len(results)) + b"".join(rs) + bytes(blob1) + bytes(blob2)


def gather_packed(local, dist, dst=0):
    """Variable-size gather of one uint8 tensor per rank to `dst`: the sizes by one all_gather,
    then every other rank sends exactly its bytes to `dst` (point-to-point, RCCL send/recv over
    xGMI with backend "nccl"; gloo on CPU) — no rank is padded to the largest.  Returns, on dst,
    the list of per-rank byte strings (rank order); None elsewhere.  `local` lives on the device
    the process group communicates on (cuda for RCCL, cpu for gloo)."""
    import torch
    world = dist.get_world_size()
    rank = dist.get_rank()
    dev = local.device
    n = torch.tensor([local.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, n)
    sz = [int(s.item()) for s in sizes]
    if rank != dst:
        if sz[rank]:
            for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, local.contiguous(), dst)]):
                w.wait()
            # with RCCL, wait() only orders torch's current stream: block the host until the send
            # has read `local`, so the caller may overwrite it (the next step's export runs on the
            # library's own stream, which is not ordered after this one)
            if dev.type == "cuda":
                torch.cuda.current_stream(dev).synchronize()
        return None
    bufs = [None] * world
    ops = []
    for r in range(world):
        if r == dst:
            bufs[r] = local
        else:
            bufs[r] = torch.empty(sz[r], dtype=torch.uint8, device=dev)
            if sz[r]:
                ops.append(dist.P2POp(dist.irecv, bufs[r], r))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return [b.cpu().numpy().tobytes() if b.numel() else b"" for b in bufs]
