"""bench.py — batched permission checks on MI355X (BASELINE.json metric, config #2).

Workload (BASELINE.json configs[1]): synthetic RBAC, 10M users, 100k
nested groups, 50M tuples, 1M checks docs:d#viewer@u per GPU (half constructed
positives), seed 0x4B45544F.  The graph is replicated on every GPU (it fits 288 GB many
times over); the global batch of N x 1M requests is split into contiguous 64-request-word
ranges, one per GPU: no data-path collective, weak scaling.  A step = one batch call over
a GPU's range with its requests already resident in HBM, enqueued without a host wait per
call (ketogpu_queries_run_async: traversal, result bits left in HBM; batches pipelined as a
server pipelines them, two HBM copies of the batch rotating over two streams) — `value`,
K steps bracketed by a barrier and a device synchronization on both sides, the max over
ranks.  Beside it: the same steps with one host wait per call (ketogpu_queries_run,
`resident_call_checks_per_s`: round 5's value) and the host-to-host rate (requests H2D from
pinned memory, traversal, result bits D2H: ketogpu_check_ids, the call SURVEY.md 8(d)
times, `host_to_host_checks_per_s`, never `value`).
Under torchrun each rank drives its own GPU; `python bench.py --gpus N` in one process
drives N GPUs through ketogpu_multi (one host thread per GPU for the resident runs).

    python bench.py [--gpus N --steps K --warmup W] [--small] [--no-cpu-baseline]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line (see the contract in README/DESIGN.md).
"""
import argparse
import json
import os
import platform
import sys
import time

import torch  # first: one HIP runtime in the process (libketogpu binds to torch's)
import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "permission checks/sec (batched, whole node) + traversal HBM GB/s vs roofline"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PIPE_COPIES = 2  # HBM copies of a GPU's batch rotating in the pipelined (value) leg


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)  # ~4 ms of resident calls: the barrier inside the timed region stays small
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--small", action="store_true", help="1/100-size graph for quick runs (not the metric)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU work of the baseline sample")
    p.add_argument("--r2-sample", type=int, default=0,
                   help="partitioned: also diff this many uniform requests of rank 0 against oracle/r2_check.c "
                        "(the independent R2 checker) fed from the same stream")
    p.add_argument("--parity", choices=["full", "sample"], default="full",
                   help="full: every request of the timed batch is diffed against the oracle (about 90 s of "
                        "16-thread CPU work at config #2); sample: only the baseline sample")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "r06", "traffic.json"),
                   help="PMC traffic summary (tools/pmc_traffic.py) for roofline.traffic")
    p.add_argument("--mode", choices=["replicated", "partitioned"], default="replicated",
                   help="replicated: graph on every GPU, request batches sharded (the metric's line); "
                        "partitioned: hash-partitioned graph, per-level all-to-all (config #5 path)")
    p.add_argument("--scale", type=float, default=0.02,
                   help="partitioned: config #5 size as a fraction of its 5B tuples (1.0 = full)")
    p.add_argument("--tier-exchange", action="store_true",
                   help="partitioned tier at world 1: run the exchange path over an RCCL communicator of one rank "
                        "(queries and replies through ncclSend/ncclRecv to itself) instead of reading rows in place")
    p.add_argument("--part-engine", choices=["tier", "level"], default="tier",
                   help="partitioned: tier = two exchanges per batch over the replicated core (ketogpu_tier_*); "
                        "level = the per-level frontier exchange (ketogpu_part_*)")
    return p.parse_args()


def dist_init(n):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def max_over_ranks(x, world):
    if world == 1:
        return x
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def kernel_source_hash():
    from keto_amd.build import kernel_source_hash as h
    return h()


def host_cores():
    """CPU threads this job may use: the scheduler affinity (= nproc), capped by a cgroup
    CPU quota when one is set (a quota of 16 CPUs on 256 visible ones runs 16 at a time)"""
    nproc = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    return (min(nproc, quota) if quota else nproc), nproc, quota


def main():
    a = parse()
    rank, world, local = dist_init(a.gpus)
    if a.mode == "partitioned":
        return main_partitioned(a, rank, world, local)
    from keto_amd import _lib as L
    from keto_amd import check, synth
    from keto_amd.snapshot import Snapshot

    # one process per GPU under torchrun (world = N), or one process driving N GPUs
    # through the replicated multi-GPU engine (world = 1, --gpus N): either way the
    # global batch of N x 1M requests is split into contiguous word ranges, one per GPU
    procs_gpus = a.gpus if world == 1 else 1
    n_gpus = world * procs_gpus
    scale = 100 if a.small else 1
    per_gpu = 1_000_000 // (10 if a.small else 1)
    sizes = dict(users=10_000_000 // scale, groups=100_000 // scale, docs=2_000_000 // scale,
                 tuples=50_000_000 // scale, checks=per_gpu * n_gpus)
    t0 = time.time()
    # every rank builds the same graph and the same global batch (same seeds)
    w = synth.rbac(**sizes, seed=synth.SEED, check_seed=synth.SEED + 1)
    t_gen = time.time() - t0
    log(f"generated {w.counts} in {t_gen:.1f}s")
    t0 = time.time()
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    t_snap = time.time() - t0
    log(f"snapshot built in {t_snap:.1f}s")
    roots_all, targets_all = w.resolve(snap)
    b, e = check.MultiEngine.ranges(len(roots_all), world)[rank]
    roots, targets = roots_all[b:e], targets_all[b:e]
    n = len(roots)
    if procs_gpus > 1:
        eng = check.MultiEngine(snap, list(range(procs_gpus)))
        eng0 = eng.engine(0)
    else:
        eng = eng0 = check.Engine(snap, device=local)
    # the batch lives in pinned host memory, as the cgo micro-batcher's buffer would
    # (ketogpu_host_alloc); results come back into pinned words
    pr, pt = check.pinned(roots), check.pinned(targets)
    words = (n + 63) // 64
    out = check.PinnedBuffer(words, np.uint64)

    def step():
        eng.check_ids_raw(pr.array.ctypes.data, pt.array.ctypes.data, n, out.array.ctypes.data)

    # plan selection (KETOGPU_UNITS=auto): each engine's first two large batches run every
    # candidate first stage and keep the fastest; done here so the timed steps never do it
    for _ in range(2):
        step()
    for _ in range(a.warmup):
        step()
    barrier(world)
    calls = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        c0 = time.perf_counter()
        step()
        calls.append(time.perf_counter() - c0)
    barrier(world)
    dt = time.perf_counter() - t0
    dt = max_over_ranks(dt, world)
    log(f"{a.steps} host-to-host steps in {dt:.4f}s")
    allowed = check.unpack_bits(out.array.copy(), n)
    host_value = len(roots_all) * a.steps / dt
    median_call = float(np.median(calls))

    # the same batch from pageable numpy arrays (no pinned staging): reported, not `value`
    c0 = time.perf_counter()
    got_pageable = eng.check_ids(roots, targets)
    t_pageable = time.perf_counter() - c0
    assert np.array_equal(got_pageable, allowed)

    # the timed step's own first-stage kernel (the host-batch instantiation reading its
    # requests from pinned memory): the same steps again with a timing event between the
    # call's kernels, hipEvents on the engine's stream (not `value`: the events cost idle
    # GPU time between the launches)
    host_runs = []
    if procs_gpus == 1:
        eng0.set_events(True)
        for _ in range(a.steps):
            step()
            host_runs.append(eng0.last_stats())
        eng0.set_events(False)
        assert np.array_equal(check.unpack_bits(out.array.copy(), n), allowed)

    # `value`: the same batch resident in HBM on every GPU of the job (uploaded before the
    # timed region; results stay in HBM), K steps between barriers + device syncs, max over
    # ranks.  One process driving several GPUs runs one host thread per GPU.
    rng = check.MultiEngine.ranges(n, procs_gpus) if procs_gpus > 1 else [(0, n)]
    engs = [eng.engine(i) for i in range(procs_gpus)] if procs_gpus > 1 else [eng0]
    qs = [e_.upload(roots[b_:e_r], targets[b_:e_r]) for e_, (b_, e_r) in zip(engs, rng)]
    for qq in qs:
        for _ in range(a.warmup + 1):
            qq.run()

    def resident(qq):
        for _ in range(a.steps):
            qq.run()
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    if len(qs) == 1:
        resident(qs[0])
    else:
        import threading
        ths = [threading.Thread(target=resident, args=(qq,)) for qq in qs]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
    torch.cuda.synchronize()
    barrier(world)
    dt_res = max_over_ranks(time.perf_counter() - t0, world)
    value = len(roots_all) * a.steps / dt_res
    log(f"{a.steps} HBM-resident steps in {dt_res:.4f}s")
    for qq, (b_, e_r) in zip(qs, rng):
        assert np.array_equal(qq.download(), allowed[b_:e_r])

    # pipelined: the same K steps enqueued without a host wait per call
    # (ketogpu_queries_run_async: the engine proves no request can need the second stage),
    # one wait per GPU at the end, barrier + device sync on both sides — batch k+1 enqueued
    # while batch k runs, as a server pipelines its batches.  PIPE_COPIES HBM copies of the
    # GPU's batch rotate (a server's consecutive batches have their own result words): calls
    # rotate over the engine's two streams, so a call's dense pass overlaps the next call's
    # first stage
    copies = [[qq] + [e_.upload(roots[b_:e_r], targets[b_:e_r]) for _ in range(PIPE_COPIES - 1)]
              for qq, e_, (b_, e_r) in zip(qs, engs, rng)]
    for cs in copies:
        for qq in cs[1:]:
            qq.run()

    def pipelined(cs, e_):
        nq = 0
        for k in range(a.steps):
            nq += cs[k % len(cs)].run(pipelined=True)
        e_.wait()
        return nq
    queued = [0] * len(qs)
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    if len(qs) == 1:
        queued[0] = pipelined(copies[0], engs[0])
    else:
        import threading

        def _p(i):
            queued[i] = pipelined(copies[i], engs[i])
        ths = [threading.Thread(target=_p, args=(i,)) for i in range(len(qs))]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
    torch.cuda.synchronize()
    barrier(world)
    dt_pipe = max_over_ranks(time.perf_counter() - t0, world)
    pipe_value = len(roots_all) * a.steps / dt_pipe
    log(f"{a.steps} pipelined HBM-resident steps in {dt_pipe:.4f}s ({sum(queued)} calls queued without a wait)")
    for cs, (b_, e_r) in zip(copies, rng):
        for qq in cs:
            assert np.array_equal(qq.download(), allowed[b_:e_r])
        for qq in cs[1:]:
            qq.close()
    b0, e0 = rng[0]
    q = qs[0]
    # the kernels' own times: the same runs again with a timing event between the call's
    # kernels (each event idles the GPU a few microseconds: not the rate above)
    eng0.set_events(True)
    runs = []
    for _ in range(a.steps):
        q.run()
        runs.append(eng0.last_stats())
    eng0.set_events(False)
    st = runs[-1]

    out_line = None
    if rank == 0:
        # per kernel family: algorithmic bytes (engine counters) / summed hipEvent time over
        # the timed HBM-resident runs
        plan = L.RunStats.PLANS.get(st["plan"], "unit")  # KETOGPU_UNITS=auto: the plan the engine kept
        # kernel families as tools/pmc_traffic.py names them (the PMC summary's keys)
        main, host_main = {
            "bidi": ("bidi_kernel<16>", "bidi_host_kernel (host batches)"),
            "lite": ("lite_kernel", "lite_host_kernel (host batches)"),
            "core": ("core lite_kernel", "core lite_host_kernel (host batches)"),
            "label": ("label_kernel", "label_host_kernel (host batches)"),
            "v2": ("unit2_kernel<16>", "unit2_kernel<16>")}.get(plan, ("unit_kernel<16>", "unit_kernel<16>"))
        tot = lambda k: sum(r[k] for r in runs)
        fam = {
            main: (tot("main_bytes"), tot("main_ms"), sum(1 for r in runs if r["main_ms"] > 0)),
            "spill stages (bidi w,q,s cascade or unit2 cascade)": (
                tot("bytes_unit") - tot("main_bytes"), tot("ms_unit") - tot("main_ms"),
                sum(max(r["unit_launches"] - 1, 0) for r in runs)),
            "expand_kernel": (tot("bytes_push"), tot("ms_push"), sum(r["push_launches"] - r["unit_launches"]
                                                                     for r in runs)),
            "pull_kernel": (tot("bytes_pull"), tot("ms_pull"), tot("rounds")),
        }
        gbps = {k: (bb / (ms * 1e-3) / 1e9 if ms > 0 else 0.0) for k, (bb, ms, _) in fam.items()}
        dominant = max(fam, key=lambda k: fam[k][1])
        traffic_doc, traffic_note = {}, "no PMC summary"
        if os.path.exists(a.traffic):
            try:
                tr = json.load(open(a.traffic))
                src_ok = tr.get("source_hash") == kernel_source_hash()
                if tr.get("workload") != ("config2_rbac" + ("_small" if a.small else "")):
                    traffic_note = "PMC summary of another workload"
                elif not src_ok:
                    traffic_note = (f"stale: {os.path.relpath(a.traffic, ROOT)} was profiled at kernel sources "
                                    f"{tr.get('source_hash')}, HEAD is {kernel_source_hash()}")
                else:
                    traffic_doc = tr.get("kernels", {})
                    traffic_note = f"{os.path.relpath(a.traffic, ROOT)} (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)"
            except (OSError, ValueError):
                traffic_note = "unreadable PMC summary"

        def roofline(name, b_k, ms_k, n_launch, requests, measured):
            ach = b_k / (ms_k * 1e-3) / 1e9 if ms_k > 0 else 0.0
            return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBPS, 4),
                    "traffic": traffic_doc.get(name, {}).get("hbm_bytes_per_launch"), "traffic_source": traffic_note,
                    "kernel": name, "bytes_per_launch": int(b_k / max(n_launch, 1)),
                    "ms_per_launch": round(ms_k / max(n_launch, 1), 4), "requests_per_launch": int(requests),
                    "measured": measured}

        # the line's roofline: the timed (HBM-resident) step's first stage; the host-to-host
        # step's own first stage beside it, with its PCIe bound
        roof = roofline(dominant, *fam[dominant], e0 - b0,
                        "hipEvents around the first stage of the HBM-resident runs (ketogpu_queries_run), "
                        "the timed steps re-run")
        if host_runs and all(r["main_ms"] > 0 for r in host_runs):
            host_roof = roofline(host_main, sum(r["main_bytes"] for r in host_runs),
                                 sum(r["main_ms"] for r in host_runs), len(host_runs), n,
                                 "hipEvents on the engine's stream around the first stage of the host-to-host "
                                 "step (ketogpu_engine_set_events), same steps re-run")
            # the same kernel against its real bound: 8 B of requests per check read over PCIe
            pcie_ach = 8 * n * len(host_runs) / (sum(r["main_ms"] for r in host_runs) * 1e-3) / 1e9
            pcie_peak = pcie_h2d_gbps(local)
            host_roof["pcie"] = {"bound": "pcie (requests read in place from pinned host memory)",
                                 "achieved": round(pcie_ach, 1), "peak": round(pcie_peak, 1), "unit": "GB/s",
                                 "peak_source": "measured: pinned 64 MiB host -> HBM DMA copy (hipMemcpyAsync)",
                                 "frac": round(pcie_ach / pcie_peak, 4) if pcie_peak > 0 else None}
            roof["host_to_host"] = host_roof
        roof["kernels"] = {k: {"GBps": round(gbps[k], 1), "ms": round(ms, 4), "bytes": bb, "launches": nl}
                           for k, (bb, ms, nl) in fam.items() if ms > 0}
        roof["line_ceiling"] = line_ceiling(local, e0 - b0, roof["ms_per_launch"])
        achieved = roof["achieved"]
        stream = stream_copy_gbps(local)
        roof["stream_copy_GBps"] = round(stream, 1)  # measured device-copy bandwidth
        roof["frac_of_stream"] = round(achieved / stream, 4) if stream > 0 else None
        cpu = None
        parity = None
        sql = None
        if not a.no_cpu_baseline and n_gpus == 1:
            cpu, parity = cpu_baseline(w, allowed, a.cpu_seconds, full=a.parity == "full")
            sql = sql_baseline(min(10.0, a.cpu_seconds))
        elif not a.no_cpu_baseline:
            # N > 1: the CPU baseline is timed at N = 1 only; rank 0's range still gets a
            # bounded parity sample against the oracle
            _, parity = cpu_baseline(w, allowed, 3.0, full=False, offset=b)
        pos = np.asarray(w.chk_pos, dtype=bool)[b:e]
        parity = dict(parity or {}, constructed_positives=int(pos.sum()),
                      constructed_positives_denied=int((pos & ~allowed.astype(bool)).sum()))
        out_line = {
            "metric": METRIC, "value": round(pipe_value, 1), "unit": "checks/s", "n_gpus": n_gpus, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(dt_pipe / a.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32 ids / u64 bitmasks (integer)",
            "data": "synthetic: config #2 RBAC generator (keto_amd/csrc/synth.cpp), seed 0x4B45544F",
            "config": {"workload": "config2_rbac" + ("_small" if a.small else ""), **sizes,
                       "checks_per_gpu": per_gpu,
                       "mode": "replicated graph, query batch split into contiguous word ranges",
                       "parallelism": (f"query-shard x{n_gpus}" + (" (one process, ketogpu_multi)" if procs_gpus > 1
                                                                 else " (one process per GPU)" if world > 1 else ""))},
            "timing": ("value: requests resident in HBM, PCIe legs excluded: per step one batch call per GPU over "
                       "its range, enqueued without a host wait per call (ketogpu_queries_run_async: validation at "
                       f"upload, traversal, result bits left in HBM; {PIPE_COPIES} HBM copies of the batch rotate, "
                       "calls rotate over the engine's two streams), one wait per GPU after the K steps, barrier + "
                       "device sync "
                       f"on both sides, max over ranks; {sum(queued)} of {a.steps * len(qs)} calls queued without a "
                       "wait; every copy's bits checked after; snapshot build and upload excluded.  SURVEY 8(d)'s "
                       "number is host_to_host_checks_per_s"),
            "resident_call_checks_per_s": round(value, 1),
            "resident_call_ms_per_step": round(dt_res / a.steps * 1e3, 4),
            "resident_call_timing": ("the same K steps with one host wait per call (ketogpu_queries_run: round 5's "
                                     "value)"),
            "host_to_host_checks_per_s": round(host_value, 1),
            "host_to_host_timing": ("ketogpu_check_ids over the GPU's range: requests H2D from pinned memory, "
                                    "traversal, result bits D2H (the call SURVEY 8(d) times); PCIe-inclusive, "
                                    "not value"),
            "host_to_host_ms_per_step": round(dt / a.steps * 1e3, 4),
            "median_call_checks_per_s": round(len(roots_all) / world / median_call, 1) if world == 1 else None,
            "call_ms": [round(c * 1e3, 4) for c in calls],
            "pageable_checks_per_s": round(n / t_pageable, 1),
            "roofline": roof, "cpu_baseline": cpu, "cpu_baseline_sql": sql, "parity": parity,
            "plan": plan + (f" ({st['plan_unit']}-request units, {st['plan_lists']}-entry lists)"
                            if plan in ("bidi", "lite", "core") else
                            f" (2-hop labels: S heads {st['label_s_head']} words, P heads {st['label_p_head']} words, "
                            f"{st['label_bytes'] / 1e9:.2f} GB)" if plan == "label" else ""),
            "engine": {k: st[k] for k in ("spilled_units", "unit_rows", "unit_edges", "unit_rev", "rounds", "levels",
                                          "frontier_entries", "interior_edges", "rev_edges", "touched", "ms_total",
                                          "hubs", "hub_build_ms", "closure_nodes_f", "closure_nodes_b",
                                          "core_build_ms", "label_on", "label_coverage", "label_build_ms",
                                          "label_pll_ms", "label_bytes", "label_entries", "label_s_head",
                                          "label_p_head")},
            # plan label's second stage (requests without labels: plan lite over the listed
            # requests): its share of the timed batch and its time (events between kernels)
            "second_stage": ({"rest_requests_per_call": [int(r["rest_requests"]) for r in host_runs] or
                              [int(st["rest_requests"])],
                              "rest_ms_per_call": [round(r["rest_ms"], 4) for r in host_runs],
                              "first_stage_ms_per_call": [round(r["main_ms"], 4) for r in host_runs],
                              "note": "rest_ms = the second stage + the statistics/emit launch, timed between "
                                      "hipEvents with KETOGPU_EVENTS between kernels"}
                             if plan == "label" else None),
            "edges_per_check": round((st["interior_edges"] + st["rev_edges"]) / max(e0 - b0, 1), 2),
            "allowed_fraction": round(float(allowed.mean()), 4),
            "setup_s": {"generate": round(t_gen, 2), "snapshot": round(t_snap, 2)},
            "snapshot": {k: v for k, v in snap.stats().items() if k.startswith("num_")},
        }
        print(json.dumps(out_line), flush=True)
    barrier(world)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def max_rss_gb():
    import resource
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6  # KB -> GB


def main_partitioned(a, rank, world, local):
    """Config #5's path (BASELINE.json configs[4]): the RBAC shape at `--scale` x 5B tuples,
    generated as a stream (synth.config5) that every rank reads in ORDER BY order while
    the partition-aware loader keeps only what the rank owns (keto_amd/partition.py Shard).
    --part-engine tier (default): the core (rows among interior nodes) gathered on every
    rank, then each rank checks ITS OWN 1M requests per step with two exchanges (seed-row
    queries and replies); level: the per-level frontier exchange over the whole batch of
    1M x world requests on every rank.  Weak scaling either way; value = the requests of
    all ranks / the slowest rank's time."""
    from keto_amd import synth
    from keto_amd.partition import Core, PartitionedEngine, Shard, TieredEngine
    import threading
    phase = ["loading the shard"]

    def heartbeat():  # long loads (minutes at --scale >= 0.1) stay visibly alive
        t_hb = time.time()
        while phase[0]:
            time.sleep(30)
            if phase[0]:
                log(f"... {phase[0]} ({time.time() - t_hb:.0f}s)")
    threading.Thread(target=heartbeat, daemon=True).start()
    f = a.scale
    sizes = dict(users=max(1000, int(500_000_000 * f)), groups=max(100, int(10_000_000 * f)),
                 docs=max(100, int(200_000_000 * f)), tuples=max(10_000, int(5_000_000_000 * f)))
    per_gpu = 1_000_000 // (10 if a.small else 1)
    n_req = per_gpu * world
    w = synth.config5(**sizes, checks=n_req, check_seed=synth.SEED + 1)
    rss0 = max_rss_gb()
    t0 = time.time()
    ncomm = None
    if a.tier_exchange and world == 1:
        from keto_amd.partition import NativeComm
        ncomm = NativeComm(device=local, kind="rccl")
    sh = Shard.load(w.namespaces, lambda: w.batches(1 << 20), native_comm=ncomm)
    t_load = time.time() - t0
    phase[0] = "building the engine, timing, parity"
    rss_load = max_rss_gb()
    sst = sh.stats()
    log(f"shard loaded in {t_load:.1f}s: {sst['rows']} rows streamed, {sst['owned_nodes']} nodes owned, "
        f"host arrays {sst['host_bytes'] / 1e9:.2f} GB, peak RSS {rss_load:.2f} GB")
    roots, targets, status = sh.resolve_batch(w.request_batch())
    from keto_amd import check
    tier = a.part_engine == "tier"
    core_info = None
    if tier:
        t0 = time.time()
        core = Core(sh, ncomm)
        cv = core.view()
        core_info = {"seconds": round(time.time() - t0, 2), "interior_nodes": int(cv["num_interior"]),
                     "forward_entries": int(len(cv["f_col"])), "backward_entries": int(len(cv["b_col"])),
                     "device_bytes": int(cv["bytes"]), "share_of_rows": round((len(cv["f_col"]) + len(cv["b_col"])) /
                                                                              max(sst["rows"], 1), 5)}
        del cv
        log(f"core gathered: {core_info}")
        eng = TieredEngine(sh, device=local, core=core, comm=ncomm)
        mine = slice(rank * per_gpu, (rank + 1) * per_gpu)  # this rank's own requests
        # resident in HBM when the timed region starts (read in place by every pass)
        dev_req = [torch.from_numpy(np.ascontiguousarray(x[mine]).view(np.int32)).to(f"cuda:{local}")
                   for x in (roots, targets)]
        torch.cuda.synchronize()
        # answers into pinned words (ketogpu_host_alloc), as the serving integration hands over
        bits_buf = check.PinnedBuffer((per_gpu + 63) // 64, np.uint64)
        bits = bits_buf.array

        def step():
            eng.check_ids_ptr(dev_req[0].data_ptr(), dev_req[1].data_ptr(), per_gpu, bits)
    else:
        # requests in pinned host memory, as for the replicated line (ketogpu_part_begin
        # copies them to HBM by DMA); every rank passes the whole batch
        pinned = (check.pinned(roots), check.pinned(targets))
        eng = PartitionedEngine(sh, device=local, record_capacity=1 << 26)

        def step():
            return eng.check_ids(pinned[0].array, pinned[1].array)
    for _ in range(max(a.warmup, 1)):  # the level engine's first call also picks the direction
        step()
    st0 = eng.stats() if tier else None
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    barrier(world)
    dt = max_over_ranks(time.perf_counter() - t0, world)
    if tier:
        got = np.unpackbits(bits.view(np.uint8), bitorder="little")[:per_gpu].astype(bool)
        st1 = eng.stats()
        d = {k: st1[k] - st0[k] for k in ("rows_opened", "records_read", "eval_kernel_ms", "eval_kernel_launches")}
        launches = max(d["eval_kernel_launches"], 1)
        tier_label = bool(st1["label"])
        if tier_label:  # list words (4 B; masks included), request ids, answer bits, list bounds
            per_req = 16 if ncomm is not None else 32  # received-list bounds, or the own lists' offsets
            bytes_launch = 4 * d["records_read"] / launches + (8 + per_req) * per_gpu + per_gpu / 8
        else:
            bytes_launch = (16 * d["rows_opened"] + 16 * d["records_read"]) / launches + 8 * per_gpu + per_gpu / 8
        ms_launch = d["eval_kernel_ms"] / launches
        achieved = bytes_launch / (ms_launch * 1e-3) / 1e9 if ms_launch > 0 else 0.0
        fam = None
        t_timed = None
    else:
        got = step()
        # measurement pass: the same step with every kernel launch bracketed by hipEvents
        before = eng.local.stats()["kernels"]
        eng.local.set_timing(True)
        t1 = time.perf_counter()
        step()
        t_timed = time.perf_counter() - t1
        eng.local.set_timing(False)
        after = eng.local.stats()
        fam = {k: {kk: after["kernels"][k][kk] - before[k][kk] for kk in ("bytes", "ms", "launches")}
               for k in after["kernels"]}
    rss = [max_rss_gb()]
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([rss[0], rss_load, float(sst["host_bytes"])], dtype=torch.float64,
                         device="cuda" if dist.get_backend() == "nccl" else "cpu")
        out_t = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out_t, t)
        per_rank = [o.tolist() for o in out_t]
    else:
        per_rank = [[rss[0], rss_load, float(sst["host_bytes"])]]
    out = None
    if rank == 0:
        if tier:
            traffic, traffic_note = None, "no PMC summary for this workload"
            kname = "tier_label_kernel" if tier_label else "tier_eval_kernel"
            tpath = os.path.join(ROOT, "profiles", "r05", f"traffic_config5_x{f:g}.json")
            if os.path.exists(tpath):  # tools/profile.sh with WORKLOAD=config5_partitioned_x<scale>
                try:
                    tr = json.load(open(tpath))
                    if tr.get("workload") != f"config5_partitioned_x{f:g}":
                        traffic_note = "PMC summary of another workload"
                    elif tr.get("source_hash") != kernel_source_hash():
                        traffic_note = (f"stale: {os.path.relpath(tpath, ROOT)} was profiled at kernel sources "
                                        f"{tr.get('source_hash')}, HEAD is {kernel_source_hash()}")
                    else:
                        traffic = tr.get("kernels", {}).get(kname, {}).get("hbm_bytes_per_launch")
                        traffic_note = f"{os.path.relpath(tpath, ROOT)} (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)"
                except (OSError, ValueError):
                    traffic_note = "unreadable PMC summary"
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                    "traffic_source": traffic_note, "kernel": kname,
                    "bytes_per_launch": int(bytes_launch), "ms_per_launch": round(ms_launch, 4),
                    "measured": "hipEvents around the first evaluation stage on the engine's stream, every timed step",
                    "bytes_formula": ("4*list words read (masks included) + 8*requests + requests/8 + 16*requests "
                                      "(received-list bounds; 32 at world 1 without exchange: the own lists' offsets)")
                                     if tier_label else
                                     "16*rows_opened + 16*records_read + 8*requests + requests/8 (as the replicated "
                                     "line's lite kernel)"}
        else:
            dominant = max(fam, key=lambda k: fam[k]["ms"])
            d = fam[dominant]
            achieved = d["bytes"] / (d["ms"] * 1e-3) / 1e9 if d["ms"] > 0 else 0.0
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
                    "traffic_source": "no PMC summary for this workload", "kernel": dominant,
                    "bytes_per_launch": int(d["bytes"] / max(d["launches"], 1)),
                    "ms_per_launch": round(d["ms"] / max(d["launches"], 1), 4),
                    "measured": "one extra step with hipEvents around every launch (ketogpu_part_set_timing)",
                    "kernels": {k: {"GBps": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1) if v["ms"] else None,
                                    "ms": round(v["ms"], 4), "bytes": v["bytes"], "launches": v["launches"]}
                                for k, v in fam.items() if v["launches"]}}
        cpu, parity = None, None
        if not a.no_cpu_baseline:
            cpu, parity = cpu_baseline_stream(w, got, a.cpu_seconds, world)
            if a.r2_sample:
                parity = dict(parity or {}, r2_check=r2_stream(w, got, a.r2_sample))
        pos = np.asarray(w.chk_pos, dtype=bool)[:len(got)]
        parity = dict(parity or {}, constructed_positives=int(pos.sum()),
                      constructed_positives_denied=int((pos & ~got.astype(bool)).sum()))
        out = {"metric": METRIC, "value": round(n_req * a.steps / dt, 1), "unit": "checks/s", "n_gpus": world,
               "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 4),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": "u32 ids / u64 bitmasks (integer)",
               "data": "synthetic: config #5 RBAC-shape stream generator (keto_amd/csrc/synth.cpp ks_c5), seed 0x4B45544F",
               "config": {"workload": f"config5_partitioned_x{f:g}", **sizes, "checks": n_req,
                          "mode": ("hash-partitioned graph (partition-aware loader), two-tier: core on every rank, "
                                   + ("2-hop label lists of the seed nodes exchanged (plan label)" if tier_label else
                                      "seed rows exchanged") + ", each rank its own requests, HBM-resident") if tier else
                                  "hash-partitioned graph (partition-aware loader), native per-level exchange",
                          "parallelism": f"partition x{world}"},
               "roofline": roof, "cpu_baseline": cpu, "parity": parity,
               "load": {"seconds": round(t_load, 1), "rows": sst["rows"], "rows_per_s": round(sst["rows"] / t_load, 1),
                        "rss_gb_before_load": round(rss0, 2),
                        "per_rank_peak_rss_gb": [round(r[0], 2) for r in per_rank],
                        "per_rank_rss_after_load_gb": [round(r[1], 2) for r in per_rank],
                        "per_rank_loader_array_gb": [round(r[2] / 1e9, 3) for r in per_rank],
                        "shard": sst}}
        if tier:
            out.update({"engine": "two-tier (ketogpu_tier_check_ids, keto_amd/csrc/tier.cpp)", "core": core_info,
                        "tier": dict(eng.stats(), exchange="RCCL grouped send/recv + all-gather"
                                     if world > 1 or ncomm is not None else "world 1: rows read in place, no exchange")})
        else:
            st = eng.local.stats()
            out.update({"engine": "per-level (ketogpu_part_check_ids, keto_amd/csrc/part_round.cpp)",
                        "partition": {k: v for k, v in st.items() if k != "kernels"},
                        "direction": {0: "forward", 1: "backward"}.get(eng.direction, "undecided"),
                        "direction_trials_ns_per_check": {{0: "forward", 1: "backward"}[k]: v
                                                          for k, v in eng._trial.items()},
                        "exchange": dict(eng.stats(), driver="native: ketogpu_part_check_ids (part_round.cpp), "
                                         "RCCL grouped send/recv + all-gather" if world > 1 else
                                         "native: ketogpu_part_check_ids (part_round.cpp), world 1: no exchange"),
                        "timed_pass_s": round(t_timed, 4)})
        print(json.dumps(out), flush=True)
    phase[0] = None
    barrier(world)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def cpu_baseline_stream(w, got, seconds, world):
    """the oracle over the streamed graph (it holds every row: only at scales one host
    holds) on the job's cores, a bounded sample of the same requests, timed at N = 1;
    its answers are the parity sample"""
    threads, nproc, quota = host_cores()
    t0 = time.time()
    from oracle import oracle as O
    st = O.Store(w.namespaces, 100)
    for cols in w.batches(1 << 20):
        st.add_columnar(cols)
    orc = st.finalize(presorted=True)
    t_build = time.time() - t0
    log(f"oracle store built in {t_build:.1f}s")
    rng = np.random.default_rng(1)
    idx = rng.permutation(len(got))
    probe = idx[:2000]
    t0 = time.perf_counter()
    orc.check_batch(w.requests(probe), nthreads=threads)
    rate = len(probe) / (time.perf_counter() - t0)
    m = int(min(len(idx), max(len(probe), rate * seconds)))
    sample = idx[:m]
    t0 = time.perf_counter()
    ans = orc.check_batch(w.requests(sample), nthreads=threads)
    ts = time.perf_counter() - t0
    mism = int((ans.astype(bool) != got[sample]).sum())
    cpu = None
    if world == 1:
        cpu = {"value": round(m / ts, 1), "unit": "checks/s", "cores": threads, "kind": "port", "nproc": nproc,
               "cgroup_cpu_quota": quota, "cpu_model": cpu_model(),
               "sample": f"{m} of the {len(got)} requests (uniform sample); oracle/keto_oracle.c over the whole "
                         f"streamed graph on {threads} threads; store build {t_build:.1f}s"}
    return cpu, {"checked": m, "of": int(len(got)), "mismatches": mism,
                 "against": "oracle/keto_oracle.c (exact restatement of internal/check/engine.go)"}


def r2_stream(w, got, m):
    """oracle/r2_check.c (its own interning, adjacency and bitset BFS; no code shared with
    libketogpu) over the same row stream, on m uniform requests of `got`"""
    from oracle import oracle as O
    threads = host_cores()[0]
    idx = np.random.default_rng(7).permutation(len(got))[:m]
    t0 = time.time()
    r2c = O.R2Checker(w.namespaces, w.requests(idx))
    for cols in w.batches(1 << 20):
        r2c.add_columnar(cols)
    build = time.time() - t0
    t0 = time.time()
    want, ok = r2c.check(nthreads=threads)
    out = {"against": "oracle/r2_check.c (independent R2 checker over the same stream)", "sample": int(ok.sum()),
           "requested": int(len(idx)), "mismatches": int((want[ok] != got[idx][ok]).sum()),
           "build_s": round(build, 1), "check_s": round(time.time() - t0, 1), "threads": threads}
    r2c.close()
    log(f"R2 checker: {out}")
    return out


def sql_baseline(seconds):
    """the reference's storage access per check — every subject-set expansion
    issues GetRelationTuples' COUNT + ORDER BY/LIMIT/OFFSET page queries (relationtuples.go:
    203-258, persister.go:106-134) against SQLite with the reference's indexes — restated in
    C through the host's libsqlite3.so.0 (oracle/keto_sql.c), one read-only connection per
    thread on every core the job may use, on a 1M-tuple graph of the config #2 generator
    (1/50 scale).  The cost regime of the reference, not the metric."""
    from keto_amd import synth
    from oracle import oracle as O
    threads, nproc, quota = host_cores()
    t0 = time.time()
    w = synth.rbac(users=200_000, groups=2_000, docs=40_000, tuples=1_000_000, checks=200_000,
                   check_seed=synth.SEED + 99)
    st = O.SqlStore(w.namespaces)
    st.add_columnar(w.columns)
    st.finish()
    t_load = time.time() - t0
    # a fixed uniform sample run to completion (per-check cost is heavy-tailed: a time
    # budget would cut the long checks and overstate the rate); the deadline only guards
    reqs = w.requests(range(min(w.n_checks, 256)))
    t0 = time.perf_counter()
    got, answered, queries = st.check_batch(reqs, nthreads=threads, seconds=max(60.0, 6 * seconds))
    dt = time.perf_counter() - t0
    done = int(answered.sum())
    # parity of the answered sample against the in-memory oracle
    sample = np.flatnonzero(answered)[:20000]
    orc = O.Store(w.namespaces, 100)
    orc.add_columnar(w.columns)
    want = orc.finalize(presorted=True).check_batch([reqs[i] for i in sample], nthreads=threads)
    mism = int((got[sample] != np.asarray(want, dtype=bool)).sum())
    st.close()
    return {"value": round(done / dt, 1), "unit": "checks/s", "cores": threads, "kind": "port-sql",
            "nproc": nproc, "cgroup_cpu_quota": quota, "sql_statements": queries,
            "statements_per_check": round(queries / max(done, 1), 1),
            "sample": f"{done} of {len(reqs)} uniform checks of a 1M-tuple config-2-shaped graph in {dt:.1f}s; every "
                      f"expansion runs the "
                      f"reference's COUNT + paged ORDER BY queries on SQLite with the reference's indexes "
                      f"(oracle/keto_sql.c through libsqlite3.so.0, {threads} threads, one connection each; db in "
                      f"tmpfs); load + index {t_load:.1f}s; {mism} mismatches vs keto_oracle.c on "
                      f"{len(sample)} of them"}


def stream_copy_gbps(device, nbytes=1 << 30, iters=10):
    """device-to-device copy bandwidth (read + write bytes / time) of a 1 GiB buffer: the
    measured ceiling beside the 8 TB/s spec"""
    a = torch.empty(nbytes, dtype=torch.uint8, device=f"cuda:{device}")
    b = torch.empty_like(a)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        b.copy_(a)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1)
    del a, b
    return 2 * nbytes * iters / (ms * 1e-3) / 1e9


def pcie_h2d_gbps(device, nbytes=64 << 20, iters=10):
    """pinned host -> HBM DMA copy bandwidth of a 64 MiB buffer: the measured PCIe ceiling
    of a host-batch first stage that reads its requests from pinned memory"""
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device=f"cuda:{device}")
    d.copy_(h, non_blocking=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        d.copy_(h, non_blocking=True)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1)
    del h, d
    return nbytes * iters / (ms * 1e-3) / 1e9


def line_ceiling(device, n, kernel_ms):
    """plan label's first stage against what its reads alone cost on this device: two random
    128-byte lines + 8 B of request per check (ketogpu_probe_random_lines, keto_amd/csrc/
    probe.hip), measured live over a 2 GiB table — the bound the HBM-byte fraction above
    cannot see (a random line costs 128 B of fetch for a 64-byte head as for a 128-byte one,
    DESIGN.md Kernels 0a)"""
    import ctypes as C
    from keto_amd import _lib as L
    ms = C.c_double(0)
    rc = L.lib().ketogpu_probe_random_lines(device, 2 << 30, n, 20, C.byref(ms))
    if rc or ms.value <= 0:
        return None
    return {"bound": "random 128-byte lines (two per check)", "probe_ms_per_launch": round(ms.value, 4),
            "kernel_ms_per_launch": kernel_ms, "frac": round(ms.value / kernel_ms, 4) if kernel_ms else None,
            "peak_lines_per_s": round(2 * n / (ms.value * 1e-3), 1),
            "achieved_lines_per_s": round(2 * n / (kernel_ms * 1e-3), 1) if kernel_ms else None,
            "measured": "ketogpu_probe_random_lines: the same request count, 16 requests per wave, both lines in "
                        "flight, 2 GiB table, hipEvents over 20 launches"}


def cpu_baseline(w, gpu_allowed, seconds, full=True, offset=0):
    """The oracle (exact restatement of the reference DFS) on every host core this job may
    use (host_cores) over a bounded sample of the same requests; its answers double as a
    bit-exact parity sample, and with `full` the rest of the batch is diffed too (SURVEY
    8(d): every timed run is checked).  gpu_allowed covers requests [offset, offset + len)."""
    from oracle import oracle as O
    from tests import randgraph
    threads, nproc, quota = host_cores()
    t0 = time.time()
    orc = randgraph.oracle_store_columns(w.namespaces, w.columns)
    t_build = time.time() - t0
    log(f"oracle store built in {t_build:.1f}s")
    rng = np.random.default_rng(1)
    idx = rng.permutation(len(gpu_allowed))
    probe = idx[:2000]
    t0 = time.perf_counter()
    ans = orc.check_batch(w.requests(probe + offset), nthreads=threads)
    tp = time.perf_counter() - t0
    rate = len(probe) / tp
    m = int(min(len(idx), max(len(probe), rate * seconds)))
    sample = idx[:m]
    t0 = time.perf_counter()
    ans = orc.check_batch(w.requests(sample + offset), nthreads=threads)
    ts = time.perf_counter() - t0
    mism = int((ans != gpu_allowed[sample]).sum())
    checked = len(sample)
    if full and m < len(idx):
        rest = idx[m:]
        t0 = time.perf_counter()
        ans_rest = orc.check_batch(w.requests(rest + offset), nthreads=threads)
        log(f"parity: remaining {len(rest)} requests diffed in {time.perf_counter() - t0:.1f}s")
        mism += int((ans_rest != gpu_allowed[rest]).sum())
        checked += len(rest)
    one = idx[:max(200, m // threads)]  # the same work on one core
    t0 = time.perf_counter()
    orc.check_batch(w.requests(one + offset), nthreads=1)
    rate1 = len(one) / (time.perf_counter() - t0)
    del O
    return ({"value": round(len(sample) / ts, 1), "unit": "checks/s", "cores": threads, "kind": "port",
             "nproc": nproc, "cgroup_cpu_quota": quota, "cpu_model": cpu_model(),
             "value_1_core": round(rate1, 1),
             "sample": f"{len(sample)} of the {len(gpu_allowed)} config-2 requests (uniform sample), full 50M-tuple "
                       f"graph; oracle/keto_oracle.c on {threads} threads (nproc {nproc}, cgroup quota {quota}) of "
                       f"{cpu_model()}; store build {t_build:.1f}s"},
            {"checked": checked, "of": int(len(gpu_allowed)), "mismatches": mism,
             "against": "oracle/keto_oracle.c (exact restatement of internal/check/engine.go)"})


if __name__ == "__main__":
    main()
