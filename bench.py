#!/usr/bin/env python3
"""Benchmark: GCUPS of 10 kbp x 10 kbp affine-gap semiglobal alignment on MI355X.

Metric (BASELINE.json): "GCUPS (billion DP cells/s), 10k x 10k affine-gap semiglobal, 1/2/4/8
MI355X".  Workload per GPU: 256 synthetic uniform-DNA pairs of 10,000 x 10,000, semiglobal,
BLOSUM62, gap open -1 / extend -2 (the reference's own config-1 parameters,
examples/from_file.rs:19-32).  One step = one pass of the hot path over the batch with the
inputs resident in HBM: DP kernel (scores + trace) -> end-cell search -> traceback writing both
aligned strings (aligner.rs:351-435).  Every rank aligns its own 256 pairs (weak scaling: the
pairs are independent, no data-path collective); after the timed region the per-rank results
are gathered to rank 0 over RCCL (reported as gather_ms).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md "HBM3E peak BW 8.0 TB/s spec"
# int32 VALU: a wave64 instruction occupies its SIMD ~4 cycles (v_max3 / v_add_sdwa / DPP measured
# 4.4 at 4 waves per SIMD, profiles/r01/micro_valu_rates.txt), i.e. 16 lanes per SIMD per cycle
VALU_PEAK_OPS = 256 * 4 * 16 * 2.4e9   # 256 CU x 4 SIMD x 16 lanes x 2.4 GHz int32 lane-ops/s
VALU_CYC_PER_INSTR = 4.4
SEED = 0xB10A11F0 + 5          # seed = 0xB10A11F0 + config index (metric = 5)


def make_pairs(npairs, n1, n2, seed):
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    pairs = []
    for _ in range(npairs):
        s1 = acgt[rng.integers(0, 4, n1)].tobytes()
        s2 = acgt[rng.integers(0, 4, n2)].tobytes()
        pairs.append((s1, s2))
    return pairs


def cpu_baseline(pairs, mode, a, b, threads):
    """The oracle (C restatement of the reference with its six full matrices) on host cores."""
    from oracle import refcpu
    secs, scores, sts = refcpu.align_batch(mode, pairs, "blosum62", a, b, nthreads=threads,
                                           exact=False)
    cells = sum(len(x) * len(y) for x, y in pairs)
    return cells / secs / 1e9, secs, scores, sts


def load_pmc(workload):
    """The committed rocprofv3 PMC summary for this workload (profiles/pmc_<workload>.json,
    written by tools/pmc_traffic.py from tools/pmc.sh passes), else {}."""
    path = os.path.join(ROOT, "profiles", "pmc_%s.json" % workload)
    if not os.path.exists(path):
        return {}
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


# Register-only ceiling of the tagged full-trace kernel's step (tools/micro/tag_step.hip on MI355X,
# 16 waves per CU, profiles/r01/micro_tag_step.txt): 5R + 2 instructions per 64R cells.
TAG_REGISTER_CEILING = {4: 6.94e12, 5: 6.60e12, 8: 7.01e12, 10: 6.94e12}


def register_ceiling(st):
    """DP cells/s if every SIMD issued the kernel's step instructions back to back at
    VALU_CYC_PER_INSTR: score-only linear step 2R + 2 instructions per 64R cells (v_add_sdwa +
    v_max3 per cell, DPP + profile address per step); tagged full trace from the micro-benchmark."""
    R = st["R"]
    if st["tagged"] and st["checkpoint"]:
        return 256 * 4 * 2.4e9 / VALU_CYC_PER_INSTR * 64 * R / (2 * R + 2), "2R+2 per 64R cells"
    if st["tagged"] and R in TAG_REGISTER_CEILING:
        return TAG_REGISTER_CEILING[R], "micro-benchmark (5R+2 per 64R cells)"
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=256)
    ap.add_argument("--len1", type=int, default=10000)
    ap.add_argument("--len2", type=int, default=10000)
    ap.add_argument("--mode", default="semiglobal")
    ap.add_argument("--open", type=int, default=-1)
    ap.add_argument("--extend", type=int, default=-2)
    ap.add_argument("--R", type=int, default=0)
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--pipeline", type=int, default=3,
                    help="slots: >= 2 lets the traceback of step k overlap the DP of step k+1 "
                         "(two HIP streams); 3 absorbs traceback times that vary around the DP's")
    ap.add_argument("--cpu-pairs", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--no-h2h", action="store_true", help="skip the host-to-host timing")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from biogarden_amd import _native

    h = _native.Handle(local_rank)
    if args.R or args.waves:
        h.set_tuning(args.R, args.waves)
    h.set_pipeline(args.pipeline)
    pairs = make_pairs(args.pairs, args.len1, args.len2, SEED + 1000003 * rank)
    sc = _native.builtin_scoring(_native.BG_BLOSUM62)
    h.prepare(args.mode, pairs, sc, args.open, args.extend)
    st = h.stats()
    cells = st["cells"]

    for _ in range(args.warmup):
        h.execute()
    h.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    h.profile_begin()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        h.execute()
    h.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    dp_ms, fin_ms, nexec = h.profile_end()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    total_cells = cells * world
    gcups = total_cells * args.steps / elapsed / 1e9

    # ---- results: RCCL gather of every rank's packed results to rank 0
    gather_ms = None
    results0 = None
    nbytes = h.export_size()
    local = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    h.export_to(local.data_ptr(), nbytes)
    if dist is not None and not args.no_gather:
        from biogarden_amd import shard
        barrier()
        tg = time.perf_counter()
        packed = shard.gather_packed(local, dist, dst=0)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - tg) * 1e3
        if rank == 0:
            results0 = [_native.decode_export(b) for b in packed]
    else:
        results0 = [_native.decode_export(local.cpu().numpy().tobytes())]

    # ---- host-to-host rate (not `value`): host buffers in, aligned strings back on the host
    h2h = None
    if not args.no_h2h:
        h.set_pipeline(1)
        torch.cuda.synchronize()
        th = time.perf_counter()
        h.prepare(args.mode, pairs, sc, args.open, args.extend)
        h.execute()
        h.fetch()
        h2h_s = time.perf_counter() - th
        h2h = {"gcups": round(cells / h2h_s / 1e9, 3), "seconds": round(h2h_s, 4),
               "covers": "bg_batch_prepare (validation, residue coding, H2D) + execute + "
                         "bg_batch_fetch (D2H of results and aligned strings), one call"}

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    ok_status = all(r["status"] == 0 for rr in results0 for r in rr)

    # ---- roofline of the DP kernel (algorithmic bytes per launch / event-timed duration)
    if st["checkpoint"]:
        # score-only DP: per lane and 64-step chunk R + 1 checkpoint ints, per strip its last row
        bytes_per_cell = (4.0 * (st["R"] + 1) + 4.0) / (64.0 * st["R"])
    else:
        bytes_per_cell = 0.25 if st["affine"] == 0 else 0.5    # the 2-bit (4-bit) trace
    algo_bytes = cells * bytes_per_cell + st["residue_bytes"]
    achieved = algo_bytes / (dp_ms * 1e-3) / 1e9 if dp_ms > 0 else 0.0
    workload = "semiglobal_%dx%dx%d_blosum62_o%d_e%d" % (args.pairs, args.len1, args.len2,
                                                          -args.open, -args.extend)
    pmc = load_pmc(workload)
    same_geom = pmc.get("geometry") == [str(st["R"]), str(st["waves"])]
    traffic = pmc.get("hbm_bytes_per_launch") if same_geom else None
    cells_per_s = cells / (dp_ms * 1e-3) if dp_ms > 0 else 0.0
    valu = {"lane_ops_peak": VALU_PEAK_OPS}
    insts = pmc.get("raw_counters", {}).get("SQ_INSTS_VALU") if same_geom else None
    if insts:
        per_cell = insts * 64.0 / cells
        valu.update({"instr_per_cell_measured": round(per_cell, 3),
                     "lane_ops_achieved": per_cell * cells_per_s,
                     "frac_of_lane_peak": round(per_cell * cells_per_s / VALU_PEAK_OPS, 4)})
    ceil_, how = register_ceiling(st)
    if ceil_:
        valu.update({"register_ceiling_cells_per_s": round(ceil_, -9), "register_ceiling_model": how,
                     "frac_of_register_ceiling": round(cells_per_s / ceil_, 4)})

    # ---- CPU baseline: the oracle on a bounded sample of the same workload (rank 0 only)
    cpu = None
    if not args.no_cpu and world == 1:
        threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)),
                             os.cpu_count() or 1))
        sample = pairs[:max(1, min(args.cpu_pairs, len(pairs)))]
        rate, secs, cscores, csts = cpu_baseline(sample, args.mode, args.open, args.extend, threads)
        gscores = [r["score"] for r in results0[0][:len(sample)]]
        cpu = {"value": round(rate, 4), "unit": "GCUPS", "cores": threads, "kind": "port",
               "sample": "%d of the %d pairs (%dx%d), oracle/refcpu.c reference-faithful full "
                         "matrices, one aligner per thread, %.1f s wall" % (
                             len(sample), len(pairs), args.len1, args.len2, secs),
               "scores_match_gpu": "%d/%d" % (sum(int(x == y) for x, y in zip(cscores, gscores)),
                                               len(sample))}

    line = {
        "metric": "GCUPS (billion DP cells/s), 10k×10k affine-gap semiglobal, 1/2/4/8 MI355X",
        "value": round(gcups, 3),
        "unit": "GCUPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (uniform DNA, numpy PCG64 seed 0x%X + 1000003*rank)" % SEED,
        "config": {"workload": workload, "pairs_per_gpu": args.pairs, "len1": args.len1,
                   "len2": args.len2, "mode": args.mode, "scoring": "blosum62",
                   "gap_open": args.open, "gap_extend": args.extend,
                   "kernel": {"R": st["R"], "waves": st["waves"], "affine": st["affine"],
                              "tagged": st["tagged"], "checkpoint": st["checkpoint"],
                              "dna_profile": st["dna"], "pipeline": args.pipeline},
                   "parallelism": "dp%d (independent pairs per rank)" % world},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "algorithmic_bytes_per_launch": int(algo_bytes),
                     "traffic_source": ("profiles/pmc_%s.json" % workload) if traffic else None,
                     "kernel": ("bg_dp_tag_kernel<ckpt>" if st["checkpoint"] else "bg_dp_tag_kernel")
                               if st["tagged"] else "bg_dp_kernel",
                     "kernel_ms": round(dp_ms, 4), "finish_ms": round(fin_ms, 4),
                     "valu": valu},
        "cpu_baseline": cpu,
        "gather_ms": None if gather_ms is None else round(gather_ms, 3),
        "host_to_host": h2h,
        "all_status_ok": ok_status,
    }
    print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
