"""bench.py — batched permission checks on MI355X (BASELINE.json metric, config #2).

Workload (BASELINE.json configs[1]): synthetic RBAC, 10M users, 100k
nested groups, 50M tuples, 1M checks docs:d#viewer@u per GPU (half constructed
positives), seed 0x4B45544F.  The graph is replicated on every GPU (it fits 288 GB many
times over) and each rank checks its own 1M requests: no data-path collective, weak
scaling.  A step = one ketogpu_queries_run over the rank's 1M HBM-resident requests.

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


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--small", action="store_true", help="1/100-size graph for quick runs (not the metric)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU work of the baseline sample")
    p.add_argument("--parity", choices=["full", "sample"], default="full",
                   help="full: every request of the timed batch is diffed against the oracle (about 90 s of "
                        "16-thread CPU work at config #2); sample: only the baseline sample")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "r01", "traffic.json"),
                   help="PMC traffic summary (tools/pmc_traffic.py) for roofline.traffic")
    p.add_argument("--mode", choices=["replicated", "partitioned"], default="replicated",
                   help="replicated: graph on every GPU, request batches sharded (the metric's line); "
                        "partitioned: hash-partitioned graph, per-level all-to-all (config #5 path)")
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


def main():
    a = parse()
    rank, world, local = dist_init(a.gpus)
    if a.mode == "partitioned":
        return main_partitioned(a, rank, world, local)
    from keto_amd import _lib as L
    from keto_amd import check, synth
    from keto_amd.snapshot import Snapshot

    scale = 100 if a.small else 1
    sizes = dict(users=10_000_000 // scale, groups=100_000 // scale, docs=2_000_000 // scale,
                 tuples=50_000_000 // scale, checks=1_000_000 // (10 if a.small else 1))
    t0 = time.time()
    # every rank builds the same graph (same seed) and draws its own 1M requests
    w = synth.rbac(**sizes, seed=synth.SEED, check_seed=synth.SEED + 1 + rank)
    t_gen = time.time() - t0
    log(f"generated {w.counts} in {t_gen:.1f}s")
    t0 = time.time()
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    t_snap = time.time() - t0
    log(f"snapshot built in {t_snap:.1f}s")
    roots, targets = w.resolve(snap)
    eng = check.Engine(snap, device=local)
    t0 = time.time()
    q = eng.upload(roots, targets)
    t_h2d = time.time() - t0

    # plan selection (KETOGPU_UNITS=auto): the engine's first two large batches run
    # both first stages and keep the faster; done here so the timed steps never do it
    for _ in range(2):
        q.run()
    for _ in range(a.warmup):
        q.run()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        q.run()
    barrier(world)
    dt = time.perf_counter() - t0
    dt = max_over_ranks(dt, world)
    log(f"{a.steps} steps in {dt:.4f}s")
    st = eng.last_stats()
    allowed = q.download()

    # PCIe-inclusive rate of one full host-to-host call (not `value`)
    t0 = time.perf_counter()
    eng.check_ids(roots, targets)
    t_host = time.perf_counter() - t0

    n = len(roots)
    value = n * world * a.steps / dt
    out = None
    if rank == 0:
        # per kernel family: algorithmic bytes (engine counters) / summed hipEvent time
        plan = L.RunStats.PLANS.get(st["plan"], "unit")  # KETOGPU_UNITS=auto: the plan the engine kept
        main = {"bidi": "bidi_kernel<16>", "v2": "unit2_kernel<16>"}.get(plan, "unit_kernel<16>")
        fam = {
            main: (st["main_bytes"], st["main_ms"], 1 if st["main_ms"] > 0 else 0),
            "spill stages (bidi w,q,s cascade or unit2 cascade)": (st["bytes_unit"] - st["main_bytes"], st["ms_unit"] - st["main_ms"],
                                                    max(st["unit_launches"] - 1, 0)),
            "expand_kernel": (st["bytes_push"], st["ms_push"], st["push_launches"] - st["unit_launches"]),
            "pull_kernel": (st["bytes_pull"], st["ms_pull"], st["rounds"]),
        }
        gbps = {k: (b / (ms * 1e-3) / 1e9 if ms > 0 else 0.0) for k, (b, ms, _) in fam.items()}
        dominant = max(fam, key=lambda k: fam[k][1])
        b_dom, ms_dom, n_launch = fam[dominant]
        achieved = gbps[dominant]
        traffic = None
        if os.path.exists(a.traffic):
            try:
                tr = json.load(open(a.traffic))
                if tr.get("workload") == ("config2_rbac" + ("_small" if a.small else "")):
                    traffic = tr.get("kernels", {}).get(dominant, {}).get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic, "kernel": dominant,
                "bytes_per_launch": int(b_dom / max(n_launch, 1)), "ms_per_launch": round(ms_dom / max(n_launch, 1), 4),
                "kernels": {k: {"GBps": round(gbps[k], 1), "ms": round(ms, 4), "bytes": b, "launches": n}
                            for k, (b, ms, n) in fam.items() if ms > 0}}
        stream = stream_copy_gbps(local)
        roof["stream_copy_GBps"] = round(stream, 1)  # measured device-copy bandwidth
        roof["frac_of_stream"] = round(achieved / stream, 4) if stream > 0 else None
        cpu = None
        parity = None
        sql = None
        if not a.no_cpu_baseline and world == 1:
            cpu, parity = cpu_baseline(w, allowed, a.cpu_seconds, full=a.parity == "full")
            sql = sql_baseline(min(10.0, a.cpu_seconds))
        elif not a.no_cpu_baseline:
            # N > 1: the CPU baseline is timed at N = 1 only; rank 0's batch still gets a
            # bounded parity sample against the oracle
            _, parity = cpu_baseline(w, allowed, 3.0, full=False)
        pos = np.asarray(w.chk_pos, dtype=bool)
        parity = dict(parity or {}, constructed_positives=int(pos.sum()),
                      constructed_positives_denied=int((pos & ~allowed.astype(bool)).sum()))
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "checks/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32 ids / u64 bitmasks (integer)",
            "data": "synthetic: config #2 RBAC generator (keto_amd/csrc/synth.cpp), seed 0x4B45544F",
            "config": {"workload": "config2_rbac" + ("_small" if a.small else ""), **sizes,
                       "checks_per_gpu": n, "mode": "replicated graph, query batches sharded",
                       "parallelism": f"query-shard x{world}"},
            "roofline": roof, "cpu_baseline": cpu, "cpu_baseline_sql": sql, "parity": parity,
            "plan": plan + (f" ({st['plan_unit']}-request units, {st['plan_lists']}-entry lists)" if plan == "bidi" else ""),
            "engine": {k: st[k] for k in ("spilled_units", "unit_rows", "unit_edges", "unit_rev", "rounds", "levels",
                                          "frontier_entries", "interior_edges", "rev_edges", "touched", "ms_total",
                                          "hubs", "hub_build_ms")},
            "edges_per_check": round((st["interior_edges"] + st["rev_edges"]) / max(n, 1), 2),
            "allowed_fraction": round(float(allowed.mean()), 4),
            "setup_s": {"generate": round(t_gen, 2), "snapshot": round(t_snap, 2), "h2d_queries": round(t_h2d, 4)},
            "pcie_inclusive_checks_per_s": round(n / t_host, 1),
            "snapshot": {k: v for k, v in snap.stats().items() if k.startswith("num_")},
        }
        print(json.dumps(out), flush=True)
    barrier(world)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def main_partitioned(a, rank, world, local):
    """Config #5's path on config #2's graph: the snapshot is hash-partitioned over the
    ranks (keto_amd/partition.py, partition.hip) and every level exchanges records with
    all_to_all over RCCL.  Every rank holds the same global batch of 1M * world requests
    (weak scaling); value = that batch / the slowest rank's time."""
    from keto_amd import check, synth
    from keto_amd.partition import PartitionedEngine
    from keto_amd.snapshot import Snapshot
    scale = 100 if a.small else 1
    n_req = (1_000_000 // (10 if a.small else 1)) * world
    sizes = dict(users=10_000_000 // scale, groups=100_000 // scale, docs=2_000_000 // scale,
                 tuples=50_000_000 // scale, checks=n_req)
    w = synth.rbac(**sizes, seed=synth.SEED, check_seed=synth.SEED + 1)
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    roots, targets = w.resolve(snap)
    eng = PartitionedEngine(snap, device=local, record_capacity=1 << 26)
    for _ in range(a.warmup):
        got = eng.check_ids(roots, targets)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        got = eng.check_ids(roots, targets)
    barrier(world)
    dt = max_over_ranks(time.perf_counter() - t0, world)
    st = eng.local.stats()
    out = None
    if rank == 0:
        # parity: the single-GPU engine on this rank's GPU holds the whole graph here
        ref = check.Engine(snap, device=local).check_ids(roots, targets)
        out = {"metric": METRIC, "value": round(n_req * a.steps / dt, 1), "unit": "checks/s", "n_gpus": world,
               "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 4),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": "u32 ids / u64 bitmasks (integer)",
               "data": "synthetic: config #2 RBAC generator, seed 0x4B45544F; graph hash-partitioned",
               "config": {"workload": "config2_rbac_partitioned" + ("_small" if a.small else ""), **sizes,
                          "mode": "hash-partitioned graph, per-level all-to-all", "parallelism": f"partition x{world}"},
               "roofline": None, "cpu_baseline": None,
               "parity": {"sample": int(n_req), "mismatches": int((got != ref).sum()),
                          "against": "single-GPU engine"},
               "partition": {k: int(v) for k, v in st.items()},
               "direction": {0: "forward", 1: "backward"}.get(eng.direction, "undecided"),
               "direction_trials_ns_per_check": {{0: "forward", 1: "backward"}[k]: v for k, v in eng._trial.items()},
               "exchange": {"records": int(eng.records), "levels": int(eng.levels), "retries": int(eng.retries)}}
        print(json.dumps(out), flush=True)
    barrier(world)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def sql_baseline(seconds):
    """the reference's storage access per check — every subject-set expansion
    issues GetRelationTuples' COUNT + ORDER BY/LIMIT/OFFSET page queries (relationtuples.go:
    203-258, persister.go:129-157) against SQLite with the reference's index — restated in
    tests/sqlite_reference.py (Python, one thread), on a 1M-tuple graph of the config #2
    generator (1/50 scale).  The cost regime of the reference, not the metric."""
    from keto_amd import persistence, synth
    from tests.sqlite_reference import SqliteReference
    t0 = time.time()
    w = synth.rbac(users=200_000, groups=2_000, docs=40_000, tuples=1_000_000, checks=20_000,
                   check_seed=synth.SEED + 99)
    c = w.columns

    def strs(name):
        data, off = c[name + "_data"].tobytes(), c[name + "_off"]
        return [data[off[i]:off[i + 1]].decode() for i in range(len(off) - 1)]
    obj, rel, sid, so, sr = (strs(k) for k in ("object", "relation", "subject_id", "ss_object", "ss_relation"))
    store = persistence.TupleStore(w.namespaces)
    kind, ns, ssns = c["subject_kind"], c["namespace_id"], c["ss_namespace_id"]
    store.conn.executemany(
        "INSERT INTO keto_relation_tuples (shard_id, nid, namespace_id, object, relation, subject_id, "
        "subject_set_namespace_id, subject_set_object, subject_set_relation, commit_time) VALUES (?,?,?,?,?,?,?,?,?,?)",
        ((str(i), store.nid, int(ns[i]), obj[i], rel[i], None if kind[i] else sid[i],
          int(ssns[i]) if kind[i] else None, so[i] if kind[i] else None, sr[i] if kind[i] else None, i)
         for i in range(len(ns))))
    ref = SqliteReference(store)
    t_load = time.time() - t0
    done = 0
    t0 = time.perf_counter()
    for q in w.requests(range(w.n_checks)):
        ref.check(q[0], q[1], q[2], ("id", q[3]["subject_id"]))
        done += 1
        if time.perf_counter() - t0 > seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": round(done / dt, 1), "unit": "checks/s", "cores": 1, "kind": "port-sql",
            "sample": f"{done} checks of a 1M-tuple config-2-shaped graph; every expansion runs the reference's "
                      f"COUNT + paged ORDER BY queries on in-memory SQLite (tests/sqlite_reference.py, Python); "
                      f"load {t_load:.1f}s"}


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


def cpu_baseline(w, gpu_allowed, seconds, full=True):
    """The oracle (exact restatement of the reference DFS) on host cores over a bounded
    sample of the same requests; its answers double as a bit-exact parity sample, and with
    `full` the rest of the batch is diffed too (every timed run is checked)."""
    from oracle import oracle as O
    from tests import randgraph
    threads = min(16, os.cpu_count() or 1)
    t0 = time.time()
    orc = randgraph.oracle_store_columns(w.namespaces, w.columns)
    t_build = time.time() - t0
    log(f"oracle store built in {t_build:.1f}s")
    rng = np.random.default_rng(1)
    idx = rng.permutation(w.n_checks)
    probe = idx[:2000]
    t0 = time.perf_counter()
    ans = orc.check_batch(w.requests(probe), nthreads=threads)
    tp = time.perf_counter() - t0
    rate = len(probe) / tp
    m = int(min(len(idx), max(len(probe), rate * seconds)))
    sample = idx[:m]
    t0 = time.perf_counter()
    ans = orc.check_batch(w.requests(sample), nthreads=threads)
    ts = time.perf_counter() - t0
    mism = int((ans != gpu_allowed[sample]).sum())
    checked = len(sample)
    if full and m < len(idx):
        rest = idx[m:]
        t0 = time.perf_counter()
        ans_rest = orc.check_batch(w.requests(rest), nthreads=threads)
        log(f"parity: remaining {len(rest)} requests diffed in {time.perf_counter() - t0:.1f}s")
        mism += int((ans_rest != gpu_allowed[rest]).sum())
        checked += len(rest)
    one = idx[:max(200, m // threads)]  # the same work on one core
    t0 = time.perf_counter()
    orc.check_batch(w.requests(one), nthreads=1)
    rate1 = len(one) / (time.perf_counter() - t0)
    del O
    return ({"value": round(len(sample) / ts, 1), "unit": "checks/s", "cores": threads, "kind": "port",
             "value_1_core": round(rate1, 1),
             "sample": f"{len(sample)} of the {w.n_checks} config-2 requests (uniform sample), full 50M-tuple graph; "
                       f"oracle/keto_oracle.c on {threads} threads of {cpu_model()}; store build {t_build:.1f}s"},
            {"checked": checked, "of": int(w.n_checks), "mismatches": mism,
             "against": "oracle/keto_oracle.c (exact restatement of internal/check/engine.go)"})


if __name__ == "__main__":
    main()
