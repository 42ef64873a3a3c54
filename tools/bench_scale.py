"""Large-graph runs of the single-GPU engine (BASELINE.json north star: >= 10^8 checks/s on
one MI355X for a 1B-tuple RBAC / folder graph).  Not the bench.py metric line: the
graph is generated and snapshotted on the host (minutes at 1B tuples), then 1M
HBM-resident requests are timed exactly as bench.py times them.

    python tools/bench_scale.py --workload rbac --tuples 1000000000
    python tools/bench_scale.py --workload folders --tuples 500000000
    python tools/bench_scale.py --workload social --tuples 1000000000

Correctness at full size: (1) every constructed positive must be allowed, (2) a uniform
sample must equal oracle/r2_check.c — an independent checker of the R2 formula over the raw
rows that shares no code with libketogpu (--r2-sample, default 20k) — (3) a sample must
equal the reference DFS restatement oracle/keto_oracle.c where it finishes within its
per-request budget (--oracle-sample; its completions and timeouts are reported), and (4) a
sample must agree with a second engine on the same snapshot running the other first stage.
A heartbeat line every 30 s keeps long host phases visibly alive.
"""
import argparse
import json
import os
import sys
import threading
import time

import torch  # noqa: F401  (one HIP runtime in the process)
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from keto_amd import check, synth  # noqa: E402
from keto_amd.snapshot import Snapshot  # noqa: E402

T0 = time.time()
PHASE = ["start"]


def log(msg):
    print(f"[scale {time.time() - T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def heartbeat():
    while True:
        time.sleep(30)
        log(f"... {PHASE[0]}")


def make(kind, tuples, checks, users=None, groups=None):
    f = tuples / {"rbac": 50e6, "folders": 500e6, "social": 1e9}[kind]
    if kind == "social" and (users or groups):  # config #4 with explicit sizes (the rows budget is `tuples`)
        return synth.social(users=users or int(100e6 * f), groups=groups or int(10e6 * f), tuples=tuples,
                            checks=checks, check_seed=synth.SEED + 1)
    if kind == "rbac":  # config #2 shape scaled: users, groups, docs grow with the tuple count
        return synth.rbac(users=int(10e6 * f), groups=int(100e3 * f), docs=int(2e6 * f), tuples=tuples, checks=checks,
                          check_seed=synth.SEED + 1)
    if kind == "folders":
        return synth.folders(users=int(10e6 * f), groups=int(100e3 * f), folders=int(20e6 * f), tuples=tuples,
                             checks=checks, check_seed=synth.SEED + 1)
    return synth.social(users=int(100e6 * f), groups=int(10e6 * f), tuples=tuples, checks=checks,
                        check_seed=synth.SEED + 1)


def rss_gb():
    import resource
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6


def mem_available():
    """bytes this process may still allocate: MemAvailable, capped by the box's per-command
    host memory limit (270 GiB) less the peak RSS so far"""
    avail = 1 << 62
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                avail = int(line.split()[1]) * 1024
    except OSError:
        pass
    return min(avail, int(270 * 2**30 - rss_gb() * 1e9))


def check_plan(k):
    from keto_amd import _lib as L
    return L.RunStats.PLANS.get(k, "unit")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", choices=["rbac", "folders", "social"], default="rbac")
    p.add_argument("--tuples", type=int, default=1_000_000_000)
    p.add_argument("--checks", type=int, default=1_000_000)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--sample", type=int, default=100_000)
    p.add_argument("--oracle-sample", type=int, default=0,
                   help="uniform requests diffed against oracle/keto_oracle.c (the whole graph is loaded into "
                        "the oracle too: host memory for two copies) and, with --expand-sample, the expand "
                        "trees of those roots diffed against the oracle's BuildTree")
    p.add_argument("--oracle-seconds", type=float, default=300.0,
                   help="bound on the oracle's check time: the sample is cut to what fits (reported)")
    p.add_argument("--oracle-request-seconds", type=float, default=20.0,
                   help="time budget per oracle request: a DFS that outlives it is counted, not waited for")
    p.add_argument("--r2-sample", type=int, default=20000,
                   help="uniform requests diffed against oracle/r2_check.c, the independent checker of the R2 "
                        "formula over the raw rows (no code shared with libketogpu); 0 = off")
    p.add_argument("--expand-sample", type=int, default=None,
                   help="BuildTree roots timed per max-depth (default 200 for folders, config #3's expand; "
                        "0 elsewhere: power-law groups expand into trees of millions of members)")
    p.add_argument("--users", type=int, default=None, help="social: users (default 100M x tuples/1e9)")
    p.add_argument("--groups", type=int, default=None, help="social: groups (default 10M x tuples/1e9)")
    a = p.parse_args()
    if a.expand_sample is None:
        a.expand_sample = 200 if a.workload == "folders" else 0
    threading.Thread(target=heartbeat, daemon=True).start()
    PHASE[0] = "generating"
    w = make(a.workload, a.tuples, a.checks, a.users, a.groups)
    t_gen = time.time() - T0
    log(f"generated {w.counts}")
    PHASE[0] = "building the snapshot"
    t0 = time.time()
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    t_snap = time.time() - t0
    st = snap.stats()
    log(f"snapshot in {t_snap:.1f}s: {st}")
    roots, targets = w.resolve(snap)
    pos = w.chk_pos.astype(bool)
    expand_roots = [q[:3] for q in w.requests(range(min(a.expand_sample, w.n_checks)))]
    orc = None
    oracle_skipped = None
    if a.oracle_sample:  # the oracle holds its own copy: ~72 B per row + the strings
        need = 72 * len(w.columns["namespace_id"]) + sum(int(w.columns[c + "_off"][-1]) + len(w.columns["namespace_id"])
                                                        for c in ("object", "relation", "subject_id", "ss_object",
                                                                  "ss_relation"))
        avail = mem_available()
        log(f"oracle store needs ~{need / 1e9:.1f} GB; available {avail / 1e9:.1f} GB; RSS {rss_gb():.1f} GB")
        if need * 1.15 > avail:
            oracle_skipped = f"oracle store needs ~{need / 1e9:.0f} GB, {avail / 1e9:.0f} GB available"
            a.oracle_sample = 0
    if a.oracle_sample:
        PHASE[0] = "building the oracle store"
        from tests import randgraph
        t0 = time.time()
        orc = randgraph.oracle_store_columns(w.namespaces, w.columns)
        log(f"oracle store in {time.time() - t0:.1f}s")
        oidx = np.random.default_rng(5).permutation(w.n_checks)[:a.oracle_sample]
        oreqs = w.requests(oidx)
    r2 = None
    if a.r2_sample:  # its own interning and adjacency of the raw rows, before they are dropped
        PHASE[0] = "building the R2 checker"
        from oracle import oracle as O
        t0 = time.time()
        ridx = np.random.default_rng(7).permutation(w.n_checks)[:a.r2_sample]
        r2c = O.R2Checker(w.namespaces, w.requests(ridx))
        r2c.add_columnar(w.columns)
        r2_build = time.time() - t0
        t0 = time.time()
        threads = min(16, os.cpu_count() or 1)
        r2_want, r2_ok = r2c.check(nthreads=threads)
        r2 = {"against": "oracle/r2_check.c (independent R2 checker: own interning, adjacency and bitset BFS over "
                         "the raw rows; pinned against keto_oracle.c in tests/test_oracle.py)",
              "sample": int(r2_ok.sum()), "requested": int(len(ridx)), "build_s": round(r2_build, 1),
              "check_s": round(time.time() - t0, 1), "threads": threads, **r2c.stats(),
              "edge_visits": int(r2c.edge_visits)}
        r2c.close()
        log(f"R2 checker: {r2}")
    del w  # the rows are no longer needed
    PHASE[0] = "uploading the device graph"
    t0 = time.time()
    eng = check.Engine(snap)
    t_up = time.time() - t0
    q = eng.upload(roots, targets)
    PHASE[0] = "timing"
    for _ in range(a.warmup):
        q.run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        q.run()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    got_sync = q.download()
    # pipelined: the same steps enqueued without a host wait per call (ketogpu_queries_run_async),
    # two HBM copies of the batch rotating over the engine's two streams
    cs = [q] + [eng.upload(roots, targets) for _ in range(1)]
    for qq in cs[1:]:
        qq.run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    queued = sum(cs[k % 2].run(pipelined=True) for k in range(a.steps))
    eng.wait()
    torch.cuda.synchronize()
    dt_pipe = time.perf_counter() - t0
    for qq in cs:
        assert np.array_equal(qq.download(), got_sync)
    for qq in cs[1:]:
        qq.close()
    eng.set_events(True)  # the first stage's own time: one more run with events between the kernels
    q.run()
    eng.set_events(False)
    rs = eng.last_stats()
    got = q.download()
    assert np.array_equal(got, got_sync)
    log(f"timed: {len(roots) * a.steps / dt:.4g} checks/s, {dt / a.steps * 1e3:.3f} ms/step, plan "
        f"{check_plan(rs['plan'])}, spilled units {rs['spilled_units']}, spilled requests {rs['spilled_requests']}, "
        f"positives denied {int((pos & ~got.astype(bool)).sum())}")
    PHASE[0] = "cross-checking"
    other = "v2" if rs["plan"] == 1 else "bidi"  # the plan the timed engine did not keep
    os.environ["KETOGPU_UNITS"] = other
    os.environ["KETOGPU_HUBS"] = "0"  # the other first stage, and no hub index: an independent evaluation
    ref_eng = check.Engine(snap)
    idx = np.random.default_rng(3).permutation(len(roots))[:a.sample]
    ref = ref_eng.check_ids(roots[idx], targets[idx])
    xmism = int((ref != got[idx]).sum())
    log(f"cross-check against the {other} engine: {xmism} mismatches of {len(idx)}")
    if r2 is not None:
        r2["mismatches"] = int((r2_want[r2_ok] != got[ridx][r2_ok]).sum())
        log(f"R2 checker parity: {r2['mismatches']} mismatches of {r2['sample']}")
    # a first result line now: a run cut short in the oracle phase still reports the timing
    print(json.dumps({"workload": f"{a.workload}_{a.tuples}", "phase": "timed", "checks": len(roots),
                      "checks_per_s": round(len(roots) * a.steps / dt, 1), "ms_per_step": round(dt / a.steps * 1e3, 4),
                      "pipelined_checks_per_s": round(len(roots) * a.steps / dt_pipe, 1),
                      "main_kernel_ms": round(rs["main_ms"], 4), "dense_pass_requests": rs["full_requests"],
                      "plan": check_plan(rs["plan"]), "positives_denied": int((pos & ~got.astype(bool)).sum()),
                      "cross_check": {"sample": int(len(idx)), "mismatches": xmism}, "r2_check": r2}), flush=True)
    oracle = None
    if orc is not None:
        PHASE[0] = "oracle sample"
        threads = min(16, os.cpu_count() or 1)
        t0 = time.perf_counter()
        mism = done = timed_out = tried = 0
        step = 4 * threads
        for k in range(0, len(oreqs), step):  # chunks under a per-request budget: nothing runs unbounded
            want, ok = orc.check_batch_budget(oreqs[k:k + step], nthreads=threads, seconds=a.oracle_request_seconds)
            sel = oidx[k:k + step]
            mism += int((want[ok] != got[sel][ok]).sum())
            done += int(ok.sum())
            timed_out += int((~ok).sum())
            tried += len(sel)
            if time.perf_counter() - t0 > a.oracle_seconds:
                break
        oracle = {"against": "oracle/keto_oracle.c", "sample": int(done), "requested": int(len(oidx)),
                  "tried": int(tried), "timed_out": int(timed_out), "request_budget_s": a.oracle_request_seconds,
                  "mismatches": mism, "seconds": round(time.perf_counter() - t0, 1), "threads": threads,
                  "oracle_checks_per_s": round(done / (time.perf_counter() - t0), 1)}
        log(f"oracle: {oracle}")
    PHASE[0] = "expand"
    from keto_amd import expand
    from keto_amd.relationtuple import SubjectSet
    xe = expand.Engine(snap)
    exp = {}
    if orc is not None and expand_roots:  # BuildTree parity: the same trees as the oracle's
        bad = 0
        for depth in (3, 5, 10):
            for ns, o, r in expand_roots:
                t = xe.BuildTree(SubjectSet(ns, o, r), depth)
                mine = t.to_node() if t else None
                want = orc.expand({"subject_set": {"namespace": ns, "object": o, "relation": r}}, depth)
                bad += mine != want
        exp["parity"] = {"against": "oracle/keto_oracle.c BuildTree", "trees": 3 * len(expand_roots),
                         "max_depths": [3, 5, 10], "mismatches": bad}
        log(f"expand parity: {exp['parity']}")
    for depth in (3, 5, 10) if expand_roots else ():  # config #3: expand at max-depth 3, 5, 10 (host DFS, R10)
        t0 = time.perf_counter()
        nodes = [xe.tree_size(SubjectSet(ns, o, r), depth) for ns, o, r in expand_roots]
        dt_e = time.perf_counter() - t0
        exp[f"max_depth_{depth}"] = {"trees_per_s": round(len(nodes) / dt_e, 1),
                                     "nodes_per_tree": round(float(np.mean(nodes)), 1), "max_nodes": int(max(nodes))}
    log(f"expand: {exp}")
    out = {"workload": f"{a.workload}_{a.tuples}", "checks": len(roots), "checks_per_s": round(len(roots) * a.steps / dt, 1),
           "ms_per_step": round(dt / a.steps * 1e3, 4),
           "pipelined_checks_per_s": round(len(roots) * a.steps / dt_pipe, 1),
           "pipelined_ms_per_step": round(dt_pipe / a.steps * 1e3, 4), "pipelined_calls_queued": int(queued),
           "main_kernel_ms": round(rs["main_ms"], 4), "dense_pass_requests": rs["full_requests"],
           "after_first_stage_ms": round(rs["rest_ms"], 4),
           "main_bytes": rs["main_bytes"], "spilled_units": rs["spilled_units"],
           "spilled_requests": rs["spilled_requests"], "allowed_fraction": round(float(got.mean()), 4),
           "constructed_positives": int(pos.sum()), "positives_denied": int((pos & ~got).sum()),
           "cross_check": {"sample": int(len(idx)), "mismatches": xmism,
                           "against": f"{other} engine without the hub index, same snapshot"},
           "parity": {"r2_check": r2, "oracle": oracle if oracle is not None else
                      ({"skipped": oracle_skipped} if oracle_skipped else None)},
           "peak_rss_gb": round(rss_gb(), 1),
           "plan": check_plan(rs["plan"]), "hubs": rs["hubs"], "hub_build_ms": round(rs["hub_build_ms"], 1),
           "core_build_ms": round(rs["core_build_ms"], 1),
           "label": ({"s_head_words": rs["label_s_head"], "p_head_words": rs["label_p_head"],
                      "bytes": rs["label_bytes"], "label_entries": rs["label_entries"],
                      "coverage": round(rs["label_coverage"], 4), "build_ms": round(rs["label_build_ms"], 1),
                      "pll_ms": round(rs["label_pll_ms"], 1), "rest_requests": rs["rest_requests"]}
                     if rs["label_on"] else None),
           "expand": dict(exp, roots=len(expand_roots), engine="host DFS over the ordered snapshot (host_engine.cpp)"),
           "setup_s": {"generate": round(t_gen, 1), "snapshot": round(t_snap, 1), "engine_upload": round(t_up, 1)},
           "snapshot": {k: v for k, v in st.items() if k.startswith("num_")}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
