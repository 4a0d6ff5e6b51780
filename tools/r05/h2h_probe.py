"""Round 5: where the streaming (host_to_host) leg's time goes.

Runs AlignStream over the metric batch with per-call host timings (collect / prepare / execute)
and prints one JSON line per variant.  --extra N opens N idle handles first (the bench's main
handle and its streams), so the stream's own streams land where the bench's do.

    python tools/r05/h2h_probe.py [--handles 4] [--pipeline 2] [--rounds 24] [--extra 1]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from tools import workloads  # noqa: E402


def run(pairs, handles, pipeline, rounds, shared):
    from biogarden_amd import _native
    from biogarden_amd.alignment import score
    from biogarden_amd.stream import AlignStream
    with AlignStream("semiglobal", score.blosum62, -1, -2, handles=handles, pipeline=pipeline,
                     raw=True, shared=shared) as st:
        for _ in range(handles):
            st.submit(pairs)
        st.drain()
        st.host_timing(reset=True)
        tcol = tprep = texe = 0.0
        texe_cpu = 0.0
        ttriv = 0.0
        from biogarden_amd._native import lib, LIB_PATH
        import ctypes
        pyexec = [ctypes.PyDLL(LIB_PATH).bg_batch_execute]
        pyexec[0].argtypes = [ctypes.c_void_p]
        t0 = time.perf_counter()
        for r in range(rounds):
            a = time.perf_counter()
            hi, ready = st._slot()
            b = time.perf_counter()
            h = st._hs[hi]
            h.set_buffer_size(*st._buf)
            h.prepare("semiglobal", pairs, score.blosum62.scoring(), -1, -2)
            st._buf = h.buffer_size()
            c = time.perf_counter()
            cc = time.thread_time()
            if PROFILE and r in (5, 6):
                evs = []
                sys.setprofile(lambda fr, ev, arg: evs.append((time.perf_counter() - c, ev, fr.f_code.co_name,
                                                               getattr(arg, "__name__", str(arg)[:40]))))
                h.execute()
                sys.setprofile(None)
                print(json.dumps({"round": r, "events": [(round(t * 1e3, 4), e, n, a) for t, e, n, a in evs]}),
                      file=sys.stderr)
            elif PYDLL:
                fn = pyexec[0]
                rc = fn(ctypes.c_void_p(h._p))
                assert rc == 0, rc
            else:
                h.execute()
            d = time.perf_counter()
            texe_cpu += time.thread_time() - cc
            e0 = time.perf_counter()
            lib().bg_group_size(None)                 # a trivial foreign call
            ttriv += time.perf_counter() - e0
            st._inflight.append((hi, r, set(), None))
            tcol += b - a
            tprep += c - b
            texe += d - c
        tdr = time.perf_counter()
        st.drain()
        t1 = time.perf_counter()
        ht = st.host_timing()
    cells = workloads.cells(pairs)
    return {"handles": handles, "pipeline": pipeline, "shared": shared,
            "gcups": round(cells * rounds / (t1 - t0) / 1e9, 1),
            "ms_per_batch": round((t1 - t0) * 1e3 / rounds, 3),
            "collect_ms": round(tcol * 1e3 / rounds, 3), "prepare_ms": round(tprep * 1e3 / rounds, 3),
            "execute_ms": round(texe * 1e3 / rounds, 3),
            "execute_thread_cpu_ms": round(texe_cpu * 1e3 / rounds, 3),
            "trivial_call_ms": round(ttriv * 1e3 / rounds, 4), "drain_ms": round((t1 - tdr) * 1e3, 3),
            "phases": {k: round(v / rounds, 3) for k, v in ht.items()}}


PROFILE = os.environ.get("H2H_PROFILE") == "1"
PYDLL = os.environ.get("H2H_PYDLL") == "1"


def cpu_stat():
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {a: int(b) for a, b in (ln.split() for ln in f)}
    except OSError:
        return {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--handles", default="4")
    ap.add_argument("--pipeline", default="2")
    ap.add_argument("--rounds", type=int, default=24)
    ap.add_argument("--extra", type=int, default=0)
    ap.add_argument("--unshared", action="store_true")
    ap.add_argument("--torch", action="store_true", help="initialise torch's HIP context first")
    ap.add_argument("--c3", action="store_true", help="run C3 on the extra handles first (WIDE streams)")
    ap.add_argument("--gcfreeze", action="store_true", help="gc.freeze() after the setup")
    args = ap.parse_args()
    from biogarden_amd import _native
    pairs = workloads.metric_pairs(256, 10000, 10000, workloads.SEED0 + 5)
    if args.torch:
        import torch
        torch.cuda.synchronize()
    extra = [_native.Handle(0) for _ in range(args.extra)]
    sc = _native.builtin_scoring(_native.BG_BLOSUM62)
    for h in extra:                       # a batch through each, so its streams exist and ran
        h.set_pipeline(3)
        h.prepare("semiglobal", pairs[:16], sc, -1, -2)
        h.execute()
        h.synchronize()
        if args.c3:
            h.prepare("semiglobal", workloads.c3_pair(), sc, -1, -2)
            for _ in range(4):
                h.execute()
            h.synchronize()
    import gc
    gct = {"n": 0, "ms": 0.0, "t": 0.0}

    def gccb(phase, info):
        if phase == "start":
            gct["t"] = time.perf_counter()
        else:
            gct["n"] += 1
            gct["ms"] += (time.perf_counter() - gct["t"]) * 1e3
    gc.callbacks.append(gccb)
    if args.gcfreeze:
        gc.collect()
        gc.freeze()
    import threading
    print(json.dumps({"python_threads": [t.name for t in threading.enumerate()],
                      "switch_interval": sys.getswitchinterval()}))
    with open("/proc/self/maps") as f:
        hip = sorted({ln.split()[-1] for ln in f if "amdhip64" in ln or "libhsa-runtime" in ln})
    print(json.dumps({"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "extra": args.extra,
                      "torch": args.torch, "c3": args.c3, "hip_libs": hip}))
    for hs in args.handles.split(","):
        for pp in args.pipeline.split(","):
            n0, ms0 = gct["n"], gct["ms"]
            cs0, t0 = cpu_stat(), os.times()
            r = run(pairs, int(hs), int(pp), args.rounds, not args.unshared)
            cs1, t1 = cpu_stat(), os.times()
            r["cgroup_cpu_stat_delta"] = {k: cs1[k] - cs0.get(k, 0) for k in cs1}
            r["process_cpu_s"] = round((t1.user + t1.system) - (t0.user + t0.system), 3)
            r["wall_s"] = round(t1.elapsed - t0.elapsed, 3)
            with open("/proc/self/status") as f:
                r["threads"] = int([x for x in f if x.startswith("Threads:")][0].split()[1])
            r["gc"] = {"collections": gct["n"] - n0, "ms": round(gct["ms"] - ms0, 2),
                       "objects": len(gc.get_objects())}
            print(json.dumps(r), flush=True)
    for h in extra:
        h.close()


if __name__ == "__main__":
    main()
