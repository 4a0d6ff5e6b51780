#!/usr/bin/env python3
"""Benchmark: GCUPS of 10 kbp x 10 kbp affine-gap semiglobal alignment on MI355X.

Metric (BASELINE.json): "GCUPS (billion DP cells/s), 10k x 10k affine-gap semiglobal, 1/2/4/8
MI355X".  Workload M per GPU: 256 synthetic uniform-DNA pairs of
10 000 x 10 000, semiglobal, BLOSUM62, gap open -1 / extend -2 (the reference's own config-1
parameters, examples/from_file.rs:19-32).  With open >= extend the Gotoh DP provably collapses to
linear gaps, so the line also carries `affine`: the same pairs with open -11 /
extend -1, the genuinely affine three-matrix DP and the reference's one-cell-late X/Y traceback.

One step = one pass of the hot path over the batch with the inputs resident in HBM: DP kernel
-> end-cell search -> traceback writing both aligned strings (aligner.rs:351-435), three
pipeline slots (the traceback of step k overlaps the DP of step k+1).

N GPUs ("the same 256 pairs are sharded over G in {1,2,4,8} (strong scaling)"):
one process per GPU.  `--gpus N` with N > 1 outside torch.distributed starts
`torch.distributed.run --nproc-per-node N` as a child before anything touches a GPU and exits
with its code; under torch.distributed the ranks must equal --gpus and (RCCL) each rank needs
a device of its own, else the bench fails.  The N > 1 headline is the strong form: ONE batch of
256 pairs LPT-sharded over the ranks, every step = execute + the device-side compact export
(bg_batch_export_compact_async, no host wait) + the RCCL gather of the records to rank 0,
pipelined, all inside the timed wall.  `weak` beside it: every rank aligns its own 256 pairs
(the record gather after the timed region).  `--weak` makes the weak form the headline.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
    ... bench.py --config C4|C5    the whole 8-GPU job of SURVEY §8(d) C4 / C5, LPT-sharded over
                                   the ranks, export + RCCL gather to rank 0 inside every step

Fields beyond the driver's contract:
  roofline        the DP kernel (the dominant one) against §8(d)'s algorithmic bytes
                  (0.25 B/cell for open >= extend, 0.5 for open < extend, plus the residues),
                  HBM peak 8 TB/s; `bound` names the roof that binds (VALU issue) and `valu`
                  its fraction: PMC-measured VALU instructions x 64 lanes / kernel time against
                  256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6e12 lane-ops/s (MI355X_MICROARCH.md)
  configs         (N = 1) the other BASELINE configurations on this GPU, each with its value,
                  step time, DP / traceback kernel times and roofline: C2, C3, and C4 / C5 as
                  one GPU's LPT share of their 8-GPU jobs
  host_to_host    PCIe-inclusive rate through the streaming API (biogarden_amd.stream): residues
                  uploaded from host buffers, aligned strings downloaded to host buffers, four
                  handles in rotation so batches' uploads and downloads overlap the kernels of
                  the batches in flight (never `value`), with the host's time per phase
  cpu_baseline    the oracle (oracle/refcpu.c: the reference's six full matrices, its loop order,
                  one reused aligner per thread) on this host's cores, plus a 1-core rate and C1
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default, and what the
# MI355X boxes' environment sets).  The bench never raises it: the streaming leg (host_to_host)
# shares one set of four streams between its handles, so it fits four queues.
HW_QUEUES_ENV = os.environ.get("GPU_MAX_HW_QUEUES")

from tools import workloads  # noqa: E402

HBM_PEAK_GBS = 8000.0                     # MI355X_MICROARCH.md "HBM3E peak BW 8.0 TB/s spec"
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9  # guide: a wave64 VALU instruction issues over 2 cycles
VALU_CYC_PER_INSTR = 4.4                   # measured issue cost of the step's v_max3 / v_add_sdwa /
                                           # DPP mix (profiles/r01/micro_valu_rates.txt)
MEASURED_ISSUE_LANE_OPS = 256 * 4 * 64 / VALU_CYC_PER_INSTR * 2.4e9
SEED = workloads.SEED0 + 5                 # seed = 0xB10A11F0 + config index (M = 5)
METRIC = "GCUPS (billion DP cells/s), 10k×10k affine-gap semiglobal, 1/2/4/8 MI355X"


def make_pairs(npairs, n1, n2, seed):
    return workloads.metric_pairs(npairs, n1, n2, seed)


# ------------------------------------------------------------------ host description


def host_info():
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity_cpus"] = os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    info["cgroup_cpu_quota"] = quota
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["cpu_model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith(("MemTotal", "MemAvailable")):
                    k, v = line.split(":")
                    info[k.strip().lower() + "_gib"] = round(int(v.split()[0]) / 2 ** 20, 1)
    except OSError:
        pass
    return info


def usable_cores(info):
    """Threads the CPU baseline runs on: every CPU this process may use (affinity), bounded by
    the cgroup's CPU quota when one is set (threads beyond it only time-share)."""
    n = info.get("affinity_cpus") or 1
    if info.get("cgroup_cpu_quota"):
        n = min(n, max(1, int(info["cgroup_cpu_quota"])))
    return max(1, n)


def cpu_baseline(pairs, mode, a, b, threads):
    """The oracle (C restatement of the reference with its six full matrices) on host cores."""
    from oracle import refcpu
    secs, scores, sts = refcpu.align_batch(mode, pairs, "blosum62", a, b, nthreads=threads,
                                           exact=False)
    return workloads.cells(pairs) / secs / 1e9, secs, scores, sts


# ------------------------------------------------------------------ PMC summaries


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


def workload_name(mode, npairs, n1, n2, a, b):
    return "%s_%dx%dx%d_blosum62_o%d_e%d" % (mode, npairs, n1, n2, -a, -b)


def kernel_name(st):
    if st.get("grouped"):
        return "bg_dp_grp_kernel<R=%d,P=%d> (%d groups of %d reads per wave)" % (
            st["R"], st["group_pairs"], st["grouped"], st["group_pairs"])
    if st["tagged"]:
        return "bg_dp_tag_kernel<R=%d,%s,ckpt=%d>" % (st["R"], "WIDE" if st["wide"] else "strips",
                                                     st["checkpoint"])
    if st["checkpoint"]:
        return "bg_dp_aff_kernel<R=%d,local=%d>" % (st["R"], st["local"])
    return "bg_dp_kernel<R=%d>" % st["R"]


def finish_name(st):
    if st.get("grouped"):
        return "bg_finish_kernel<R=%d,checkpoint,grouped P=%d>" % (st["R"], st["group_pairs"])
    if st.get("split"):
        return "split traceback (bg_exit_kernel<R=%d> + bg_finish_kernel phases)" % st["R"]
    return "bg_finish_kernel<R=%d,%s>" % (st["R"], "checkpoint" if st["checkpoint"] else "trace")


def roofline(st, cells, dp_ms, workload, a, b, fin_ms=None):
    """§8(d): algorithmic bytes per cell 0.25 (open >= extend: 2-bit m_trace) or 0.5 (4-bit trace)
    plus the residues, over the event-timed launch of the step's DOMINANT kernel: the DP, or the
    traceback stream when it runs longer (its kernels' time on their stream); VALU from the PMC
    summary (the DP's)."""
    bpc = 0.25 if a >= b else 0.5
    algo = cells * bpc + st["residue_bytes"]
    fin_dom = fin_ms is not None and fin_ms > dp_ms
    dom_ms = fin_ms if fin_dom else dp_ms
    achieved = algo / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    pmc = load_pmc(workload)
    same = pmc.get("geometry") == [str(st["R"]), str(st["waves"])]
    traffic = pmc.get("hbm_bytes_per_launch") if same else None
    cps = cells / (dp_ms * 1e-3) if dp_ms > 0 else 0.0
    valu = {"peak_lane_ops_per_s": VALU_PEAK_LANE_OPS,
            "peak_source": "MI355X_MICROARCH.md: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz"}
    insts = pmc.get("raw_counters", {}).get("SQ_INSTS_VALU") if same else None
    if insts:
        ipc = insts * 64.0 / cells
        valu.update({"instr_per_cell": round(ipc, 3),
                     "lane_ops_per_s": round(ipc * cps, -9),
                     "frac": round(ipc * cps / VALU_PEAK_LANE_OPS, 4),
                     # second figure: against the measured ~4.4-cycle issue of this mix
                     "frac_of_measured_issue": round(ipc * cps / MEASURED_ISSUE_LANE_OPS, 4),
                     "pmc_source": "profiles/pmc_%s.json" % workload})
    return {"bound": "valu", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic if not fin_dom else None,
            "frac_basis": "HBM roofline of SURVEY 8(d): (%.2f B/cell + residues) / the dominant "
                          "kernel's time / 8 TB/s; the binding roof is VALU issue (see valu.frac)" % bpc,
            "algorithmic_bytes_per_launch": int(algo),
            "traffic_source": ("profiles/pmc_%s.json" % workload) if (traffic and not fin_dom) else None,
            "kernel": finish_name(st) if fin_dom else kernel_name(st),
            "kernel_ms": round(dom_ms, 4), "dominant": "traceback" if fin_dom else "dp",
            "dp_kernel": kernel_name(st), "dp_ms": round(dp_ms, 4), "valu": valu}


# ------------------------------------------------------------------ timed runs


def timed(h, steps, warmup, barrier, per_step=None):
    """K executes between barriers; `per_step` (the export + gather of a sharded job) runs after
    every execute, inside the timed region."""
    for _ in range(warmup):
        h.execute()
        if per_step:
            per_step()
    h.synchronize()
    barrier()
    h.profile_begin()
    t0 = time.perf_counter()
    for _ in range(steps):
        h.execute()
        if per_step:
            per_step()
    h.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    dp_ms, fin_ms, _ = h.profile_end()
    return elapsed, dp_ms, fin_ms


def gatherer(h, dist, coll_dev, stats=None):
    """Per-step §8(e) result path: bg_batch_export_compact packs the last execute's headers and
    alignment cores (2-bit edit scripts) device-to-device, then one variable-size gather to rank 0
    (RCCL send/recv over xGMI; gloo rehearsal on host tensors).  Returns a callable -> rank 0:
    list of per-rank records (bytes); `stats` (dict) receives the payload bytes."""
    import torch
    from biogarden_amd import shard
    buf = {"t": None}

    def step():
        n = h.export_compact_size()
        if buf["t"] is None or buf["t"].numel() < n:
            buf["t"] = torch.empty(max(n, 1), dtype=torch.uint8, device="cuda")
        h.export_compact_to(buf["t"].data_ptr(), n)
        src = buf["t"][:n]
        if stats is not None:
            stats["record_bytes"] = n
        if dist is None:
            return [src.cpu().numpy().tobytes()]
        return shard.gather_packed(src if coll_dev == "cuda" else src.cpu(), dist, dst=0)
    return step


def sharded_job(pairs, mode, a, b, world, rank):
    """LPT shard of one batch (shard.lpt_shards, balanced by cells) with the per-pair scratch
    dims a single reference aligner would start each call from (shard.call_dims)."""
    from biogarden_amd import shard
    sizes = [(len(x), len(y)) for x, y in pairs]
    shards = shard.lpt_shards(sizes, world)
    mine = shards[rank]
    return [pairs[p] for p in mine], shard.shard_call_dims(mode, sizes, a, b, mine), shards


def host_to_host(pairs, mode, a, b, device, rounds=8, pipeline=2, handles=4, shared=True):
    """PCIe-inclusive throughput through the product's streaming API (biogarden_amd.stream.
    AlignStream): per batch the residues are staged from host buffers (validation, pinned
    staging, H2D), the kernels run, and the aligned strings come back into host buffers; the
    stream's handle rotation keeps `handles` batches in flight so uploads, downloads and the
    host's byte passes overlap the kernels.  The handles share one set of four HIP streams
    (uploads, DPs, tracebacks, downloads), so the leg fits the box's 4 hardware queues.  This is
    SURVEY §8(d)'s wall: H2D of the residues, DP, end cell, traceback and the strings on the
    host."""
    from biogarden_amd.alignment import score
    from biogarden_amd.stream import AlignStream
    with AlignStream(mode, score.blosum62, a, b, device=device, handles=handles,
                     pipeline=pipeline, raw=True, shared=shared) as st:
        for _ in range(handles):                       # warm every handle's arenas
            st.submit(pairs)
        st.drain()
        st.host_timing(reset=True)
        t0 = time.perf_counter()
        done = 0
        for r in range(rounds):
            done += len(st.submit(pairs, tag=r))
        done += len(st.drain())
        secs = time.perf_counter() - t0
        ht = st.host_timing()
    assert done == rounds
    cells = workloads.cells(pairs)
    # per batch: the host is one thread through the rotation, so its phases add up to the wall;
    # `other` is Python, the launches and the waits outside prepare / fetch
    phases = {k: round(v / rounds, 4) for k, v in ht.items()
              if k not in ("prepares", "fetches", "host_threads")}
    phases["other"] = round(secs * 1e3 / rounds - sum(phases.values()), 4)
    return {"gcups": round(cells * rounds / secs / 1e9, 2), "rounds": rounds, "handles": handles,
            "seconds_per_batch": round(secs / rounds, 5),
            "host_ms_per_batch": phases, "host_threads": int(ht.get("host_threads", 0)),
            "prepares": int(ht.get("prepares", 0)), "fetches": int(ht.get("fetches", 0)),
            "streams": 4 if shared else 3 * handles, "shared_streams": shared,
            "covers": "biogarden_amd.stream.AlignStream: bg_batch_prepare (validation, pinned "
                      "staging, H2D) + execute + the strings' download queued behind the "
                      "traceback (bg_download_kernel writing host-mapped pinned buffers) + "
                      "bg_batch_fetch (aligned strings in host buffers), %d handles in rotation "
                      "on %s" % (handles, "one shared set of 4 HIP streams" if shared
                                 else "streams of their own"),
            "survey_8d_wall": True}


def cpu_section(pairs, gpu_scores, mode, a, b, info, pairs_multi, pairs_one):
    """Rank 0 at N = 1: the oracle on every usable core over a bounded sample of M, on 1 core
    over >= 8 pairs, and C1 (the reference's own example) on 1 core."""
    threads = usable_cores(info)
    nm = min(len(pairs), max(pairs_multi, threads))
    sample = pairs[:nm]
    rate, secs, cscores, _ = cpu_baseline(sample, mode, a, b, threads)
    one = pairs[:pairs_one]
    rate1, secs1, cs1, _ = cpu_baseline(one, mode, a, b, 1)
    out = {"value": round(rate, 4), "unit": "GCUPS", "cores": threads, "kind": "port",
           "sample": "%d of the %d M pairs (10000x10000), oracle/refcpu.c reference-faithful "
                     "(six full matrices, 15 B/cell), one reused aligner per thread, %d threads, "
                     "%.1f s wall" % (nm, len(pairs), threads, secs),
           "scores_match_gpu": "%d/%d" % (sum(int(x == y) for x, y in zip(cscores, gpu_scores)), nm),
           "one_core": {"value": round(rate1, 4), "pairs": len(one), "seconds": round(secs1, 2),
                        "scores_match_gpu": "%d/%d" % (
                            sum(int(x == y) for x, y in zip(cs1, gpu_scores)), len(one))},
           "host": info}
    try:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from conftest import REF_FIX, read_fasta
        recs = read_fasta(os.path.join(REF_FIX, "input", "semiglobal_alignment.fasta"))
        c1 = [(recs[0][1], recs[1][1])]
        r1, s1_, sc1, _ = cpu_baseline(c1, "semiglobal", -1, -2, 1)
        out["C1_one_core"] = {"value": round(r1, 4), "seconds": round(s1_, 3), "score": sc1[0],
                              "cells": workloads.cells(c1),
                              "config": "semiglobal_alignment.fasta 9559x8457, blosum62 -1/-2"}
        # C3 (100 kbp x 100 kbp) on the CPU needs the reference's 150 GB of matrices and ~80 s:
        # too long for this line; extrapolated from C1's in-run 1-core rate, with the measured
        # run of tools/c3_cpu.py on an MI355X box beside it (strings equal to the GPU's)
        c3 = {"extrapolated_seconds": round(1e10 / (r1 * 1e9), 1),
              "basis": "1e10 cells at this run's C1 one-core rate"}
        try:
            with open(os.path.join(ROOT, "profiles", "r03", "c3_cpu.json")) as f:
                m = json.loads(f.read())
            c3["measured_record"] = {"file": "profiles/r03/c3_cpu.json", "seconds": m.get("cpu_seconds"),
                                     "gcups_one_core": m.get("cpu_gcups_one_core"),
                                     "strings_equal_gpu": m.get("strings_equal")}
        except (OSError, ValueError):
            pass
        out["C3_one_core"] = c3
    except (OSError, IndexError, ImportError):
        pass
    return out


def kernel_info(st, pipeline):
    return {"R": st["R"], "waves": st["waves"], "affine": st["affine"], "tagged": st["tagged"],
            "checkpoint": st["checkpoint"], "wide": st["wide"], "split": st.get("split", 0),
            "dna_profile": st["dna"],
            "pipeline": pipeline, "fin_waves": st["fin_waves"], "fin_slots": st["fin_slots"],
            "grouped": st.get("grouped", 0), "group_pairs": st.get("group_pairs", 0)}


# K for the configs legs: the metric's default (20) for every configuration, so that each leg's
# last traceback (outside any overlap, inside the timed region) weighs the same 1/K in all of them
CONFIG_STEPS = {"C2": 20, "C3": 20, "C4": 20, "C5": 20}


def config_leg(h, sc, name, barrier, pipeline, steps=None):
    """One SURVEY §8(d) configuration on this GPU (N = 1): C2 / C3 whole, C4 / C5 as rank 0's
    LPT share of their 8-GPU jobs (with the whole job's call history for status 4)."""
    mode, pairs, a, b = workloads.job(name)
    job_cells = workloads.cells(pairs)
    share = None
    if name in ("C4", "C5"):
        pairs, dims, shards = sharded_job(pairs, mode, a, b, 8, 0)
        h.set_call_dims(dims)
        share = "rank 0 of 8 (LPT by cells): %d of %d pairs, %.4g of %.4g cells" % (
            len(pairs), sum(len(x) for x in shards), workloads.cells(pairs), job_cells)
    h.prepare(mode, pairs, sc, a, b)
    st = h.stats()
    k = steps or CONFIG_STEPS[name]
    el, dp, fin = timed(h, k, 2, barrier)
    res = h.fetch_raw()
    steady = None
    if el / k < 2e-3:
        # short steps: 20 of them (~26 ms for C4) land anywhere in a 7 300 - 10 000 GCUPS spread,
        # while 200-step runs settle at one rate per process: reported beside value
        ks = 200
        el_s, dp_s, fin_s = timed(h, ks, 2, barrier)
        steady = {"steps": ks, "value": round(st["cells"] * ks / el_s / 1e9, 3),
                  "ms_per_step": round(el_s / ks * 1e3, 4), "dp_ms": round(dp_s, 4),
                  "finish_ms": round(fin_s, 4)}
    roof = roofline(st, st["cells"], dp, name, a, b, fin)
    roof["finish_ms"] = round(fin, 4)
    single = None
    if name == "C3":
        # SURVEY 8(d)'s wall of ONE alignment: execute + synchronize, nothing in flight before it
        walls, dps, fins = [], [], []
        for _ in range(5):
            h.synchronize()
            t0 = time.perf_counter()
            h.execute()
            h.synchronize()
            walls.append((time.perf_counter() - t0) * 1e3)
            s2 = h.stats()
            dps.append(s2["dp_ms"])
            fins.append(s2["finish_ms"])
        med = sorted(walls)[len(walls) // 2]
        single = {"wall_ms": round(med, 4), "wall_ms_min": round(min(walls), 4),
                  "dp_ms": round(sorted(dps)[2], 4), "traceback_ms": round(sorted(fins)[2], 4),
                  "value": round(st["cells"] / (med * 1e-3) / 1e9, 3), "unit": "GCUPS", "runs": 5,
                  "covers": "one bg_batch_execute (DP, end cell, traceback, strings) + synchronize, "
                            "median of 5"}
        if st.get("split"):
            single["split_stats"] = h.split_stats()
    out = {"workload": workloads.DESCRIPTION[name], "pairs": len(pairs), "cells": st["cells"],
           "share": share, "value": round(st["cells"] * k / el / 1e9, 3), "unit": "GCUPS",
           "steps": k, "ms_per_step": round(el / k * 1e3, 4), "dp_ms": round(dp, 4),
           "finish_ms": round(fin, 4), "kernel": kernel_info(st, pipeline), "roofline": roof,
           "all_status_ok": all(x in (0, 4) for x in res["status"]),
           "status4": sum(1 for x in res["status"] if x == 4), "single": single,
           "steady_state": steady}
    if single is not None:
        # C3 is ONE alignment (BASELINE configs[2]): its value is that alignment's wall; executes
        # re-aligning the pair back to back (two DP streams side by side) are reported apart
        out["back_to_back"] = {"value": out["value"], "ms_per_step": out["ms_per_step"],
                               "steps": k, "covers": "%d executes of the pair pipelined" % k}
        out["value"] = single["value"]
        out["ms_per_step"] = single["wall_ms"]
        out["value_covers"] = "one alignment: execute + synchronize wall, median of 5 (single)"
    return out

# ------------------------------------------------------------------ N ranks


def spawn_ranks(argv, n):
    """--gpus N > 1 outside torch.distributed: N ranks under torch.distributed.run as a CHILD
    process, started before this process touches a GPU (no HIP call has run here); returns the
    child's exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + argv
    return subprocess.call(cmd)


class StrongGather:
    """The per-step result path of the strong form, with no host wait: the last
    execute's compact record goes into a device buffer of its own (bg_batch_export_compact_async,
    torch's current stream made to wait for it), then one gather of the fixed-capacity records
    to rank 0 (RCCL send / recv queued on that stream; every rank's capacity is exchanged once).
    Buffers rotate over `ring` steps; a buffer is reused only after the event recorded behind
    its gather.  With gloo (the CPU rehearsal) the record is copied to the host first."""

    def __init__(self, h, dist, coll_dev, ring=8):
        import torch
        self.h, self.dist, self.coll_dev = h, dist, coll_dev
        self.cap = h.export_compact_bound()
        self.caps = [self.cap]
        if dist is not None:
            t = torch.tensor([self.cap], dtype=torch.int64, device=coll_dev)
            caps = [torch.zeros(1, dtype=torch.int64, device=coll_dev) for _ in range(dist.get_world_size())]
            dist.all_gather(caps, t)
            self.caps = [int(c.item()) for c in caps]
        self.rank = 0 if dist is None else dist.get_rank()
        self.ring = ring
        self.send = [torch.empty(self.cap, dtype=torch.uint8, device="cuda") for _ in range(ring)]
        self.recv = None
        if self.rank == 0 and dist is not None:
            self.recv = [[torch.empty(c, dtype=torch.uint8, device=coll_dev) for c in self.caps]
                         for _ in range(ring)]
        self.done = [None] * ring
        self.i = 0
        self.last = None

    def __call__(self):
        import torch
        k = self.i % self.ring
        self.i += 1
        if self.done[k] is not None:
            self.done[k].synchronize()
        buf = self.send[k]
        stream = torch.cuda.current_stream()
        self.h.export_compact_async(buf.data_ptr(), self.cap, stream.cuda_stream)
        dist = self.dist
        if dist is None:
            self.last = [buf]
        else:
            src = buf if self.coll_dev == "cuda" else buf.cpu()
            if self.rank == 0:
                bufs = self.recv[k]
                ops = [dist.P2POp(dist.irecv, bufs[r], r) for r in range(1, len(bufs))]
                bufs[0] = src
            else:
                ops = [dist.P2POp(dist.isend, src, 0)]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            self.last = bufs if self.rank == 0 else None
        ev = torch.cuda.Event()
        ev.record(stream)
        self.done[k] = ev

    def records(self):
        """rank 0: the last step's records (bytes, trimmed to their own size), rank order."""
        import struct
        if self.last is None:
            return None
        out = []
        for b in self.last:
            raw = b.cpu().numpy().tobytes()
            _, n, ops, _ = struct.unpack_from("<4Q", raw, 0)
            out.append(raw[:32 + 48 * n + ops])
        return out


def dry_line(args, world, rank, dist):
    """--dry-run (no GPU): the N-rank plumbing alone — the ranks torch.distributed.run started,
    the LPT shards of one batch, a per-pair record of each rank's shard (index, lengths, CRC32 of
    both sequences) gathered to rank 0 with the same variable-size gather, merged in caller order
    and compared with the same records made for the whole batch in one process.  No alignment
    runs: `value` is null."""
    import zlib

    import torch
    from biogarden_amd import shard
    pairs = make_pairs(args.pairs, args.len1, args.len2, SEED)
    sizes = [(len(x), len(y)) for x, y in pairs]
    shards = shard.lpt_shards(sizes, world)

    def rec(p):
        return (p, len(pairs[p][0]), len(pairs[p][1]), zlib.crc32(pairs[p][0]), zlib.crc32(pairs[p][1]))

    mine = shards[rank]
    blob = json.dumps([rec(p) for p in mine]).encode()
    if dist is not None:
        packed = shard.gather_packed(torch.frombuffer(bytearray(blob), dtype=torch.uint8), dist, dst=0)
    else:
        packed = [blob]
    if rank != 0:
        return
    per = [[tuple(r) for r in json.loads(b.decode())] for b in packed]
    merged = shard.merge_shards(shards, per)
    single = [rec(p) for p in range(len(pairs))]
    print(json.dumps({"metric": METRIC, "value": None, "unit": "GCUPS", "dry_run": True,
                      "ranks": world, "n_gpus": 0, "devices": [], "gpus_arg": args.gpus,
                      "pairs": len(pairs), "shard_pairs": [len(x) for x in shards],
                      "shard_cells": [sum(sizes[p][0] * sizes[p][1] for p in x) for x in shards],
                      "gathered_pairs": sum(len(x) for x in per),
                      "gather_equals_single": merged == single,
                      "covers": "torch.distributed.run children, LPT shards, variable-size gather "
                                "to rank 0, merge in caller order; no GPU work"}))



def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pairs", type=int, default=256)
    ap.add_argument("--len1", type=int, default=10000)
    ap.add_argument("--len2", type=int, default=10000)
    ap.add_argument("--mode", default="semiglobal")
    ap.add_argument("--open", type=int, default=-1)
    ap.add_argument("--extend", type=int, default=-2)
    ap.add_argument("--affine-open", type=int, default=-11)
    ap.add_argument("--affine-extend", type=int, default=-1)
    ap.add_argument("--R", type=int, default=0)
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--pipeline", type=int, default=3,
                    help="slots: >= 2 lets the traceback of step k overlap the DP of step k+1 "
                         "(two HIP streams); 3 absorbs traceback times that vary around the DP's")
    ap.add_argument("--weak", action="store_true",
                    help="N > 1: the weak form (own --pairs per rank) as the headline instead of "
                         "the strong form (one batch of --pairs LPT-sharded over the ranks)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: the N-rank plumbing only (spawn, shards, gather, merge), value null")
    ap.add_argument("--config", choices=["C2", "C3", "C4", "C5"],
                    help="headline = this whole SURVEY 8(d) job LPT-sharded over the ranks, "
                         "export + gather to rank 0 inside every step")
    ap.add_argument("--configs", default="C2,C3,C4,C5",
                    help="N = 1: configurations timed beside M ('' for none)")
    ap.add_argument("--cpu-pairs", type=int, default=32, help="M pairs for the all-core CPU rate")
    ap.add_argument("--cpu-one-pairs", type=int, default=8, help="M pairs for the 1-core CPU rate")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-affine", action="store_true")
    ap.add_argument("--no-steady", action="store_true", help="skip the 200-step steady-state timing")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--no-h2h", action="store_true", help="skip the host-to-host timing")
    ap.add_argument("--h2h-handles", type=int, default=4,
                    help="handles (batches in flight) in the host-to-host rotation")
    ap.add_argument("--h2h-unshared", action="store_true",
                    help="host-to-host handles on streams of their own (round-4 layout, A/B)")
    ap.add_argument("--h2h-rounds", type=int, default=48,
                    help="timed batches of the host-to-host leg (the stream's fill and drain, "
                         "~one batch's latency, spread over them)")
    ap.add_argument("--group", action="store_true",
                    help="one process drives --gpus devices through the C ABI's bg_group (LPT "
                         "shards, compact export, RCCL gather to device 0, host expansion): every "
                         "step is one bg_group_align_batch of --pairs x N pairs, host to host")
    ap.add_argument("--group-devices", default="",
                    help="--group members as device ids (a device may repeat: virtual shards), "
                         "default 0..N-1")
    args = ap.parse_args()

    # N ranks: one process per GPU.  Outside torch.distributed, --gpus N > 1 starts the N ranks
    # as a child (before anything here touches a GPU) and exits with its code; inside it, the
    # ranks must be what --gpus asks for
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None and not args.group:
        sys.exit(spawn_ranks(sys.argv[1:], args.gpus))
    world = int(world_env or "1")
    if world != args.gpus and not args.group:
        print("bench.py: %d ranks under torch.distributed but --gpus %d" % (world, args.gpus),
              file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    # BG_BENCH_BACKEND=gloo rehearses the N > 1 path with ranks sharing devices (collectives on
    # host tensors; the line says how many devices ran); the driver's runs use RCCL, one GPU per rank
    backend = "gloo" if args.dry_run else os.environ.get("BG_BENCH_BACKEND", "nccl")
    coll_dev = "cuda" if backend == "nccl" else "cpu"

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
        dry_line(args, world, rank, dist)
        if dist is not None:
            dist.destroy_process_group()
        return
    ndev = torch.cuda.device_count()          # no HIP initialisation on this image
    if world > 1:
        if ndev < 1 or (backend == "nccl" and ndev < local_world):
            print("bench.py: %d ranks on this node need %d GPUs, %d visible (BG_BENCH_BACKEND=gloo "
                  "rehearses with ranks sharing devices)" % (local_world, local_world, ndev),
                  file=sys.stderr)
            sys.exit(3)
        local_rank = local_rank % ndev
        torch.cuda.set_device(local_rank)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    # the devices that ran: (host, PCI bus id) of every rank's GPU
    props = torch.cuda.get_device_properties(local_rank)
    me = (os.uname().nodename, "%s:%s" % (getattr(props, "pci_domain_id", 0), getattr(props, "pci_bus_id", local_rank)))
    if dist is not None:
        everyone = [None] * world
        dist.all_gather_object(everyone, me)
    else:
        everyone = [me]
    n_devices = len(set(everyone))
    if backend == "nccl" and n_devices != world:
        print("bench.py: %d ranks ran on %d distinct GPUs" % (world, n_devices), file=sys.stderr)
        sys.exit(3)
    if n_devices < world:
        # ranks sharing a GPU (the gloo rehearsal): WIDE and SPAN DPs spin on workgroups of their
        # own grid, and two processes' grids on one GPU could each hold part of the CUs forever
        os.environ["BG_OPTIONS"] = ",".join(x for x in (os.environ.get("BG_OPTIONS", ""), "span=0,wide=0") if x)

    from biogarden_amd import _native

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(x):
        if dist is None:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t)
        return float(t.item())

    if args.group:
        group_line(args)
        return

    h = _native.Handle(local_rank)
    if args.R or args.waves:
        h.set_tuning(args.R, args.waves)
    h.set_pipeline(args.pipeline)
    sc = _native.builtin_scoring(_native.BG_BLOSUM62)

    args.n_devices = n_devices
    if args.config:
        job_line(args, h, sc, world, rank, dist, coll_dev, barrier, max_over_ranks, sum_over_ranks)
        return

    # ---- M: the metric workload.  N = 1: the 256 pairs.  N > 1: the strong form (one batch of
    # 256 pairs LPT-sharded, export + gather in every step) and the weak form (own 256 per rank)
    workload = workload_name(args.mode, args.pairs, args.len1, args.len2, args.open, args.extend)
    own = make_pairs(args.pairs, args.len1, args.len2, SEED + 1000003 * rank)   # rank 0: the batch
    strong_head = world > 1 and not args.weak

    def weak_leg(hh):
        hh.prepare(args.mode, own, sc, args.open, args.extend)
        st_ = hh.stats()
        el, dp, fin = timed(hh, args.steps, args.warmup, barrier)
        return st_, max_over_ranks(el), dp, fin, sum_over_ranks(st_["cells"])

    def strong_leg(hh):
        spairs, sdims, shards = sharded_job(make_pairs(args.pairs, args.len1, args.len2, SEED),
                                            args.mode, args.open, args.extend, world, rank)
        hh.set_call_dims(sdims)
        hh.prepare(args.mode, spairs, sc, args.open, args.extend)
        st_ = hh.stats()
        g = None if args.no_gather else StrongGather(hh, dist, coll_dev)
        el, dp, fin = timed(hh, args.steps, args.warmup, barrier, g)
        return st_, max_over_ranks(el), dp, fin, sum_over_ranks(st_["cells"]), g, spairs, shards

    gather_ms = None
    heads0 = None
    gstats = {}
    strong = weak = None
    expand_check = None
    if strong_head:
        st, elapsed, dp_ms, fin_ms, total_cells, g, pairs, shards = strong_leg(h)
        if g is not None and rank == 0:
            recs = g.records()
            heads0 = [_native.compact_headers(b) for b in recs]
            # rank 0 expands the last step's gathered records into aligned strings (it holds the
            # inputs): the merged batch must be complete, in caller order, every status 0
            batch = make_pairs(args.pairs, args.len1, args.len2, SEED)
            te = time.perf_counter()
            per = [_native.expand_compact(rec, [batch[p] for p in idx]) for rec, idx in zip(recs, shards)]
            from biogarden_amd import shard as _shard
            merged = _shard.merge_shards(shards, per)
            expand_check = {"pairs": len(merged), "complete": all(r is not None for r in merged),
                            "expand_ms": round((time.perf_counter() - te) * 1e3, 2),
                            "covers": "rank 0, bg_compact_expand of the last step's gathered "
                                      "records (after the timed steps)"}
    else:
        st, elapsed, dp_ms, fin_ms, total_cells = weak_leg(h)
        pairs = own
    cells = st["cells"]
    gcups = total_cells * args.steps / elapsed / 1e9
    ms_per_step = elapsed / args.steps * 1e3
    # not `value`: the same batch over 200 steps, where the first DP (no traceback beside it) and
    # the last traceback (nothing beside it) weigh 1/200 instead of 1/K
    steady = None
    if not strong_head and not args.no_steady:
        ks = 200
        el_s, dp_s, fin_s = timed(h, ks, 2, barrier)
        el_s = max_over_ranks(el_s)
        steady = {"steps": ks, "value": round(total_cells * ks / el_s / 1e9, 3),
                  "ms_per_step": round(el_s / ks * 1e3, 4), "dp_ms": round(dp_s, 4),
                  "finish_ms": round(fin_s, 4)}
    roof = roofline(st, cells, dp_ms, workload, args.open, args.extend, fin_ms)
    roof["finish_ms"] = round(fin_ms, 4)
    if strong_head:
        roof["share"] = "rank 0's LPT share: %d of %d pairs" % (len(pairs), args.pairs)

    # ---- the other form beside the headline (N > 1)
    if world > 1 and strong_head:
        wst, wel, wdp, wfin, wtotal = weak_leg(h)
        weak = {"value": round(wtotal * args.steps / wel / 1e9, 3), "unit": "GCUPS",
                "ms_per_step": round(wel / args.steps * 1e3, 4), "pairs_per_rank": len(own),
                "dp_ms": round(wdp, 4), "finish_ms": round(wfin, 4), "scaling": "weak",
                "gather_in_wall": False, "kernel": kernel_info(wst, args.pipeline)}
    elif world > 1:
        hs = _native.Handle(local_rank)
        hs.set_pipeline(args.pipeline)
        sst, se, sdp, sfin, scells, _, spairs, _ = strong_leg(hs)
        strong = {"value": round(scells * args.steps / se / 1e9, 3), "unit": "GCUPS",
                  "ms_per_step": round(se / args.steps * 1e3, 4), "pairs_total": args.pairs,
                  "pairs_this_rank": len(spairs), "dp_ms": round(sdp, 4), "finish_ms": round(sfin, 4),
                  "gather_in_wall": True, "scaling": "strong", "kernel": kernel_info(sst, args.pipeline)}
        hs.close()

    # ---- results of the weak form: RCCL gather of every rank's packed results to rank 0 after
    # the timed region (the strong form gathered inside every step); N = 1: the export alone
    if not strong_head:
        if dist is not None and not args.no_gather:
            gfun = gatherer(h, dist, coll_dev, gstats)
            barrier()
            tg = time.perf_counter()
            packed = gfun()
            torch.cuda.synchronize()
            gather_ms = (time.perf_counter() - tg) * 1e3
            if rank == 0:
                heads0 = [_native.compact_headers(b) for b in packed]
        else:
            heads0 = [_native.compact_headers(b) for b in gatherer(h, None, coll_dev, gstats)()]
    if weak is not None and rank == 0:
        weak["gather_ms"] = gather_ms

    # ---- MA: the same pairs with a genuinely affine gap model (open < extend)
    aff = None
    if not args.no_affine:
        a2, b2 = args.affine_open, args.affine_extend
        h.prepare(args.mode, own, sc, a2, b2)
        sta = h.stats()
        na = max(2, args.steps // 2)
        ea, dpa, fina = timed(h, na, max(1, args.warmup // 2), barrier)
        ea = max_over_ranks(ea)
        resa = h.fetch_raw()
        wla = workload_name(args.mode, args.pairs, args.len1, args.len2, a2, b2)
        ra = roofline(sta, sta["cells"], dpa, wla, a2, b2, fina)
        ra["finish_ms"] = round(fina, 4)
        aff = {"workload": wla, "value": round(sum_over_ranks(sta["cells"]) * na / ea / 1e9, 3),
               "unit": "GCUPS", "steps": na, "ms_per_step": round(ea / na * 1e3, 4),
               "gap_open": a2, "gap_extend": b2, "kernel": kernel_info(sta, args.pipeline),
               "roofline": ra, "all_status_ok": all(s == 0 for s in resa["status"])}

    # ---- the other BASELINE configurations on this GPU (N = 1)
    cfgs = None
    if world == 1 and args.configs:
        cfgs = {}
        for name in [c for c in args.configs.split(",") if c]:
            cfgs[name] = config_leg(h, sc, name, barrier, args.pipeline)

    # ---- host-to-host rate (not `value`): host buffers in, aligned strings back on the host
    h2h = None
    if not args.no_h2h:
        queues = int(os.environ.get("GPU_MAX_HW_QUEUES") or 4)
        h2h = host_to_host(own, args.mode, args.open, args.extend, local_rank,
                           handles=args.h2h_handles, rounds=args.h2h_rounds,
                           shared=not args.h2h_unshared)
        h2h["hw_queues"] = queues
        h2h["hw_queues_source"] = "environment" if HW_QUEUES_ENV else "HIP default (unset)"

    if rank != 0:
        h.close()
        if dist is not None:
            dist.destroy_process_group()
        return

    ok_status = heads0 is not None and all(x == 0 for rr in heads0 for x, _, _ in rr)
    if expand_check is not None:
        ok_status = ok_status and expand_check["complete"]
    gpu_scores = [x for _, x, _ in heads0[0]] if heads0 else []

    # ---- CPU baseline: the oracle on a bounded sample of the same workload (rank 0, N = 1)
    cpu = None
    if not args.no_cpu and world == 1:
        cpu = cpu_section(own, gpu_scores, args.mode, args.open, args.extend, host_info(),
                          args.cpu_pairs, args.cpu_one_pairs)

    line = {
        "metric": METRIC,
        "value": round(gcups, 3),
        "unit": "GCUPS",
        "n_gpus": n_devices,
        "ranks": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong_head else "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (uniform DNA, numpy PCG64 seed 0x%X%s)" % (
            SEED, "" if strong_head else " + 1000003*rank"),
        "config": {"workload": workload, "pairs_total": args.pairs if strong_head else args.pairs * world,
                   "pairs_this_rank": len(pairs), "len1": args.len1,
                   "len2": args.len2, "mode": args.mode, "scoring": "blosum62",
                   "gap_open": args.open, "gap_extend": args.extend,
                   "kernel": kernel_info(st, args.pipeline),
                   "parallelism": "dp%d (%s)" % (world, "one batch LPT-sharded over the ranks, "
                                                 "compact export + RCCL gather to rank 0 in every "
                                                 "step" if strong_head
                                                 else "independent pairs per rank")},
        "devices": sorted(set("%s/%s" % d for d in everyone)),
        "rehearsal": None if n_devices == world else "ranks share %d GPU(s): WIDE / SPAN plans off" % n_devices,
        "collectives": backend if world > 1 else None,
        "roofline": roof,
        "steady_state": steady,
        "cpu_baseline": cpu,
        "affine": aff,
        "strong": strong,
        "weak": weak,
        "gathered_expand": expand_check,
        "configs": cfgs,
        "gather_ms": None if gather_ms is None else round(gather_ms, 3),
        "gather_record_bytes_per_rank": gstats.get("record_bytes"),
        "host_to_host": h2h,
        # SURVEY §8(d) defines GCUPS over a wall that includes H2D, traceback and the strings on
        # the host: that is host_to_host (value is the build contract's HBM-resident rate)
        "survey_8d_wall_gcups": None if h2h is None else h2h["gcups"],
        "all_status_ok": ok_status,
    }
    print(json.dumps(line))
    h.close()
    if dist is not None:
        dist.destroy_process_group()


def group_line(args):
    """--group: the multi-device path of the C ABI in ONE process (bg_group_align_batch, the
    binding a Rust caller of INTEGRATION.md uses).  Each step aligns --pairs x members pairs of M
    from host buffers to host strings: LPT split over the members, per-member prepare / execute /
    compact export on host threads, RCCL send / recv to the first member's device, one download,
    host expansion (SURVEY 8(d)'s wall; per-device work fixed as N grows: weak)."""
    import ctypes
    from biogarden_amd import _native
    devs = ([int(x) for x in args.group_devices.split(",") if x] if args.group_devices
            else list(range(args.gpus)))
    pairs = []
    for m in range(len(devs)):
        pairs += make_pairs(args.pairs, args.len1, args.len2, SEED + 1000003 * m)
    sc = _native.builtin_scoring(_native.BG_BLOSUM62)
    g = _native.Group(devs)
    try:
        for _ in range(max(1, args.warmup)):
            g.align_batch_raw(args.mode, pairs, sc, args.open, args.extend)
        # synchronous calls (bg_group_align_batch), a few
        nsync = max(2, args.steps // 4)
        t0 = time.perf_counter()
        for _ in range(nsync):
            g.align_batch_raw(args.mode, pairs, sc, args.open, args.extend)
        el_sync = time.perf_counter() - t0
        # the value: three batches in flight (bg_group_submit / bg_group_collect), every batch
        # collected into host strings inside the timed region
        # the caller's result buffers rotate (three batches in flight), as a streaming caller's
        # would; written once before timing so their pages are in
        tot = sum(len(x) + len(y) for x, y in pairs)
        bufs = [((_native.BgPairResult * len(pairs))(), (ctypes.c_uint8 * tot)(), (ctypes.c_uint8 * tot)())
                for _ in range(3)]
        for bset in bufs:
            t = g.submit(args.mode, pairs, sc, args.open, args.extend)
            g.collect(t, bset)
        g.timing(reset=True)
        t0 = time.perf_counter()
        tickets = []
        bad = 0                      # pairs of any collected batch with a status other than 0
        for s in range(args.steps):
            if len(tickets) == 3:
                res, _, _ = g.collect(tickets.pop(0), bufs[(s - 3) % 3])
                bad += sum(1 for p in range(len(pairs)) if res[p].status != 0)
            tickets.append(g.submit(args.mode, pairs, sc, args.open, args.extend))
        s = args.steps
        while tickets:
            res, _, _ = g.collect(tickets.pop(0), bufs[(s - len(tickets) - 1) % 3])
            bad += sum(1 for p in range(len(pairs)) if res[p].status != 0)
        el = time.perf_counter() - t0
        ph = g.timing()
    finally:
        g.close()
    cells = workloads.cells(pairs)
    calls = max(1, ph.pop("calls"))
    line = {"metric": METRIC, "value": round(cells * args.steps / el / 1e9, 3), "unit": "GCUPS",
            "pipelined": 3, "synchronous": {"value": round(cells * nsync / el_sync / 1e9, 3),
                                            "ms_per_call": round(el_sync / nsync * 1e3, 4),
                                            "calls": nsync},
            "n_gpus": len(set(devs)), "members": devs, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int32",
            "data": "synthetic (uniform DNA, numpy PCG64 seed 0x%X + 1000003*member)" % SEED,
            "config": {"workload": workload_name(args.mode, args.pairs, args.len1, args.len2,
                                                 args.open, args.extend),
                       "pairs_per_member": args.pairs, "mode": args.mode,
                       "parallelism": "bg_group over %d member(s) in one process: LPT shards, "
                                      "compact export, RCCL gather to device %d, host expansion; "
                                      "three batches in flight (submit / collect)"
                                      % (len(devs), devs[0])},
            "host_ms_per_step": {k: round(v / calls, 4) for k, v in ph.items()},
            "survey_8d_wall": True,
            "all_status_ok": bad == 0, "status_checked": "every collected batch"}
    print(json.dumps(line))


def job_line(args, h, sc, world, rank, dist, coll_dev, barrier, max_over_ranks, sum_over_ranks):
    """--config C2..C5: the whole SURVEY §8(d) job LPT-sharded over the ranks (§8(e)); every
    step = execute + device export + gather to rank 0 (RCCL), so the wall is §8(d)'s."""
    import torch
    from biogarden_amd import _native
    name = args.config
    mode, allp, a, b = workloads.job(name)
    pairs, dims, shards = sharded_job(allp, mode, a, b, world, rank)
    h.set_call_dims(dims)
    h.prepare(mode, pairs, sc, a, b)
    st = h.stats()
    gstats = {}
    g = gatherer(h, dist, coll_dev, gstats)
    steps = args.steps
    el, dp, fin = timed(h, steps, args.warmup, barrier, g)
    el = max_over_ranks(el)
    total = sum_over_ranks(st["cells"])
    # the same job without the per-step gather (executes pipelined back to back)
    el2, _, _ = timed(h, steps, 1, barrier)
    el2 = max_over_ranks(el2)
    packed = g()
    roof = roofline(st, st["cells"], dp, name, a, b, fin)
    roof["finish_ms"] = round(fin, 4)
    if rank == 0:
        from biogarden_amd import shard
        # rank 0 expands every rank's edit scripts into the aligned strings (it holds the inputs)
        te = time.perf_counter()
        per = [_native.expand_compact(rec, [allp[p] for p in idx]) for rec, idx in zip(packed, shards)]
        expand_ms = (time.perf_counter() - te) * 1e3
        merged = shard.merge_shards(shards, per)
        line = {"metric": "GCUPS (billion DP cells/s), %s, %d MI355X" % (name, world),
                "value": round(total * steps / el / 1e9, 3), "unit": "GCUPS",
                "n_gpus": args.n_devices, "ranks": world,
                "steps": steps, "warmup": args.warmup, "ms_per_step": round(el / steps * 1e3, 4),
                "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
                "dtype": "int32", "data": "synthetic (tools/workloads.py, seed 0xB10A11F0 + %s)" % name[1:],
                "config": {"workload": workloads.DESCRIPTION[name], "pairs": len(allp),
                           "cells": int(total), "kernel": kernel_info(st, args.pipeline),
                           "parallelism": "dp%d (whole job LPT-sharded by cells, export + "
                                          "gather to rank 0 in every step)" % world},
                "pipelined_no_gather": {"value": round(total * steps / el2 / 1e9, 3),
                                        "ms_per_step": round(el2 / steps * 1e3, 4)},
                "gather_record_bytes_rank0": gstats.get("record_bytes"),
                "expand_ms": round(expand_ms, 2),
                "expand_covers": "rank 0, bg_compact_expand of every rank's record into aligned "
                                 "strings (host, after the timed steps)",
                "roofline": roof,
                "all_status_ok": all(r is not None and r["status"] in (0, 4) for r in merged)}
        print(json.dumps(line))
    h.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
