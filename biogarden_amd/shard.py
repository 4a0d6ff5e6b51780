"""Multi-GPU plumbing for batches of independent pairs.

One process per GPU.  A batch is split over ranks by cells (largest-first greedy, like the
in-GPU pair plan); every rank runs its shard through its own `bg_aligner`, packs the results
on the device with `bg_batch_export`, and rank 0 collects the packed records with one
variable-size gather (RCCL over xGMI with backend "nccl", gloo on CPU).  No collective is on
the data path: the pairs share nothing (reference: one `SequenceAligner` call per pair,
src/alignment/aligner.rs:84-435).
"""
import struct

from . import _native


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
    """Variable-size gather of one uint8 tensor per rank to `dst`.  Returns, on dst, the list of
    per-rank byte strings (rank order); None elsewhere.  `local` lives on the device the
    process group communicates on (cuda for RCCL, cpu for gloo)."""
    import torch
    world = dist.get_world_size()
    dev = local.device
    n = torch.tensor([local.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, n)
    mx = int(max(int(s.item()) for s in sizes))
    buf = torch.zeros(max(mx, 1), dtype=torch.uint8, device=dev)
    buf[:local.numel()] = local
    gl = [torch.empty_like(buf) for _ in range(world)] if dist.get_rank() == dst else None
    dist.gather(buf, gl, dst=dst)
    if dist.get_rank() != dst:
        return None
    return [g[:int(s.item())].cpu().numpy().tobytes() for g, s in zip(gl, sizes)]
