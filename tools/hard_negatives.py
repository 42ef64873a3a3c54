"""Config #4's hard negatives against the reference DFS (VERDICT r03 "next round" 3).

At 1.0e9 rows of the power-law graph (BASELINE config #4) a negative check walks a closure
of ~10^6 groups, so a uniform oracle sample finishes only the easy requests.  Two runs
(each inside one gpurun time limit):

    python tools/hard_negatives.py pick   OUT.json [--tuples 1e9 --users 125e6 --candidates 20000 --keep 64]
        generate the graph; the independent R2 checker (oracle/r2_check.c) over a uniform
        candidate sample of the bench's requests reports each request's answer and the size
        of its root's interior closure X(r); keep the negatives with the largest closures;
        the engine (default plan, whole graph on the GPU) answers them; write indices,
        answers and closure sizes
    python tools/hard_negatives.py oracle OUT.json RESULT.json [--budget 120]
        generate the same graph; oracle/keto_oracle.c (the reference's recursion restated)
        answers the kept requests under a per-request time budget on every job core; diff
        against the engine's and the R2 checker's answers; report finished / tried

The graph and the requests are the generator's (seeded), so both runs see the same
requests without moving the rows between boxes.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_scale import make  # noqa: E402

T0 = time.time()


def log(msg):
    print(f"[hard {time.time() - T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def heartbeat(phase):
    while True:
        time.sleep(30)
        log(f"... {phase[0]}")


def threads():
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, min(os.cpu_count() or 1, int(int(q) // int(period))))
    except (OSError, ValueError):
        pass
    return min(16, os.cpu_count() or 1)


def pick(a, phase):
    import torch  # noqa: F401  (one HIP runtime in the process)
    from keto_amd import check
    from keto_amd.snapshot import Snapshot
    from oracle import oracle as O
    phase[0] = "generating"
    w = make("social", a.tuples, 1_000_000, a.users, a.groups)
    log(f"generated {w.counts}")
    phase[0] = "R2 checker"
    cand = np.sort(np.random.default_rng(11).permutation(w.n_checks)[:a.candidates])
    r2c = O.R2Checker(w.namespaces, w.requests(cand))
    r2c.add_columnar(w.columns)
    want, ok = r2c.check(nthreads=threads())
    size = r2c.closure_size.copy()
    r2c.close()
    neg = np.flatnonzero(ok & ~want)
    order = neg[np.argsort(-size[neg].astype(np.int64), kind="stable")][:a.keep]
    keep = cand[order]
    log(f"R2: {int((ok & ~want).sum())} negatives of {len(cand)}; kept closures {int(size[order].min())}.."
        f"{int(size[order].max())} nodes (median over all negatives {int(np.median(size[neg]))})")
    phase[0] = "snapshot"
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    roots, targets = w.resolve(snap)
    w_rows = w.counts["tuples"]
    del w
    phase[0] = "engine"
    eng = check.Engine(snap)
    for _ in range(2):  # the auto plan's trials, then the kept plan
        got_all = eng.check_ids(roots, targets)
    st = eng.last_stats()
    got = got_all[keep]
    out = {"tuples": a.tuples, "users": a.users, "groups": a.groups, "rows": int(w_rows), "candidates": int(len(cand)), "keep": keep.tolist(),
           "closure_size": size[order].astype(int).tolist(), "r2_answer": want[order].astype(int).tolist(),
           "engine_answer": got.astype(int).tolist(), "engine_plan": int(st["plan"]),
           "engine_vs_r2_mismatches": int((got != want[order]).sum()),
           "candidate_negatives": int((ok & ~want).sum()),
           "median_negative_closure": int(np.median(size[neg]))}
    json.dump(out, open(a.out, "w"), indent=1)
    log(f"engine vs R2 on the kept negatives: {out['engine_vs_r2_mismatches']} mismatches; plan {out['engine_plan']}")


def oracle(a, phase):
    from oracle import oracle as O
    from tests import randgraph
    picked = json.load(open(a.out))
    phase[0] = "generating"
    w = make("social", picked["tuples"], 1_000_000, picked.get("users"), picked.get("groups"))
    log(f"generated {w.counts}")
    assert w.counts["tuples"] == picked.get("rows", w.counts["tuples"]), "not the picked graph"
    phase[0] = "oracle store"
    orc = randgraph.oracle_store_columns(w.namespaces, w.columns)
    keep = np.asarray(picked["keep"], dtype=np.int64)
    reqs = w.requests(keep)
    del w
    phase[0] = "oracle checks"
    nt = threads()
    t0 = time.perf_counter()
    ans = np.zeros(len(keep), dtype=bool)
    done = np.zeros(len(keep), dtype=bool)
    for k in range(0, len(keep), nt):  # one request per core, every chunk under the budget
        a_, ok_ = orc.check_batch_budget(reqs[k:k + nt], nthreads=nt, seconds=a.budget)
        ans[k:k + nt], done[k:k + nt] = a_[:len(reqs[k:k + nt])], ok_[:len(reqs[k:k + nt])]
        log(f"oracle chunk {k // nt}: {int(ok_.sum())} of {len(reqs[k:k + nt])} finished")
        if time.perf_counter() - t0 > a.seconds:
            break
    eng = np.asarray(picked["engine_answer"], dtype=bool)
    r2 = np.asarray(picked["r2_answer"], dtype=bool)
    tried = int(min(len(keep), (k // nt + 1) * nt))
    res = {"against": "oracle/keto_oracle.c (internal/check/engine.go:33-95 restated)",
           "graph": f"config #4 power-law, {picked.get('rows', picked['tuples']):.4g} rows"
                    + (f", {picked['users']} users" if picked.get("users") else ""), "threads": nt,
           "request_budget_s": a.budget, "tried": tried, "finished": int(done.sum()),
           "timed_out": int(tried - done.sum()),
           "mismatches_vs_engine": int((ans[done] != eng[done]).sum()),
           "mismatches_vs_r2": int((ans[done] != r2[done]).sum()),
           "finished_negatives": int((done & ~ans).sum()),
           "closure_size_finished": [int(x) for x in np.asarray(picked["closure_size"])[done]],
           "seconds": round(time.perf_counter() - t0, 1),
           "picked_from": {k: picked[k] for k in ("candidates", "candidate_negatives", "median_negative_closure",
                                                  "engine_plan", "engine_vs_r2_mismatches")}}
    json.dump(res, open(a.result, "w"), indent=1)
    log(f"result: {res}")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("cmd", choices=["pick", "oracle"])
    p.add_argument("out")
    p.add_argument("result", nargs="?")
    p.add_argument("--tuples", type=float, default=1e9)
    p.add_argument("--candidates", type=int, default=20000)
    p.add_argument("--keep", type=int, default=64)
    p.add_argument("--users", type=int, default=125_000_000,
                   help="125M users x 10M groups: the generator's 1.0e9-row shape (its default 100M gives 8.1e8 rows)")
    p.add_argument("--groups", type=int, default=10_000_000)
    p.add_argument("--budget", type=float, default=120.0)
    p.add_argument("--seconds", type=float, default=560.0, help="stop starting oracle chunks after this")
    a = p.parse_args()
    a.tuples = int(a.tuples)
    phase = ["start"]
    threading.Thread(target=heartbeat, args=(phase,), daemon=True).start()
    pick(a, phase) if a.cmd == "pick" else oracle(a, phase)


if __name__ == "__main__":
    main()
