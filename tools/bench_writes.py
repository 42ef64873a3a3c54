"""Write-path freshness at config #2 scale: what an in-place write
costs on a writable snapshot, what the free slots cost the checks, and that the engine
answers like a rebuilt one afterwards.

    python tools/bench_writes.py [--tuples 50000000] [--sizes 1,10,100,1000,10000]

Steps: the config #2 RBAC graph (synth.rbac) is built twice — compact and writable
(KETOGPU_BUILD_WRITABLE) — and 1M requests are timed on both (HBM-resident, as bench.py's
hbm leg, and host to host from pinned memory, as bench.py's value).  Then write batches of
each size (half group-membership inserts — existing and new users — half deletes of
existing membership rows) go through ketogpu_snapshot_write + ketogpu_engine_sync; every
inserted membership must be allowed right after its write (read-your-writes).  Finally
the compact snapshot gets the same batches through ketogpu_snapshot_apply (the rebuild
path, timed) and a request sample — the config's requests plus every written pair — must
agree bit for bit between the written engine and the rebuilt one.
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime in the process)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from keto_amd import check, synth  # noqa: E402
from keto_amd.relationtuple import InternalRelationTuple, SubjectID  # noqa: E402
from keto_amd.snapshot import Snapshot  # noqa: E402

T0 = time.time()


def log(msg):
    print(f"[writes {time.time() - T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def timed_hbm(eng, roots, targets, steps=5):
    q = eng.upload(roots, targets)
    for _ in range(3):  # the first two runs of >= 65536 requests are the plan trials
        q.run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        q.run()
    torch.cuda.synchronize()
    return len(roots) * steps / (time.perf_counter() - t0)


def timed_host(eng, roots, targets, steps=5):
    n = len(roots)
    r, t = check.pinned(roots), check.pinned(targets)
    a = check.PinnedBuffer((n + 63) // 64, np.uint64)
    eng.check_ids_raw(r.p, t.p, n, a.p)
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.check_ids_raw(r.p, t.p, n, a.p)
    return n * steps / (time.perf_counter() - t0)


def membership_rows(cols, k, rng):
    """k random existing groups:g#member@u rows"""
    ns, kind = cols["namespace_id"], cols["subject_kind"]
    cand = np.flatnonzero((ns == 1) & (kind == 0))
    pick = cand[rng.integers(0, len(cand), size=k)]
    s = lambda c, i: bytes(cols[c + "_data"][cols[c + "_off"][i]:cols[c + "_off"][i + 1]]).decode()
    return [(1, s("object", i), s("relation", i), s("subject_id", i), None, None, None) for i in pick]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--tuples", type=int, default=50_000_000)
    p.add_argument("--sizes", default="1,10,100,1000,10000")
    p.add_argument("--sample", type=int, default=100_000)
    p.add_argument("--nest", type=int, default=20, help="nesting rows written last (the interior graph changes)")
    p.add_argument("--relabel-permille", type=int, default=None,
                   help="KETOGPU_LABEL_RELABEL_PERMILLE for the writable engine (e.g. 2: the nesting write crosses "
                        "it and starts a background relabel, timed to its swap)")
    a = p.parse_args()
    if a.relabel_permille is not None:
        os.environ["KETOGPU_LABEL_RELABEL_PERMILLE"] = str(a.relabel_permille)
    f = a.tuples / 50e6
    w = synth.rbac(users=int(10e6 * f), groups=int(100e3 * f), docs=int(2e6 * f), tuples=a.tuples, checks=1_000_000,
                   check_seed=synth.SEED + 1)
    log(f"generated {w.counts}")
    out = {"workload": f"config2_rbac_{a.tuples}", "checks": w.n_checks}
    t0 = time.time()
    compact = Snapshot.from_columns(w.namespaces, w.columns)
    out["build_s"] = {"compact": round(time.time() - t0, 1)}
    t0 = time.time()
    wsnap = Snapshot.from_columns(w.namespaces, w.columns, writable=True)
    out["build_s"]["writable"] = round(time.time() - t0, 1)
    gc, gw = compact.graph(), wsnap.graph()
    out["device_entries"] = {"compact": {"fint": int(gc["fint_off"][-1]), "rev": int(gc["rev_off"][-1])},
                             "writable": {"fint": int(gw["fint_off"][-1]), "rev": int(gw["rev_off"][-1])}}
    log(f"snapshots built {out['build_s']}, device entries {out['device_entries']}")
    roots, targets = w.resolve(compact)
    wroots, wtargets = w.resolve(wsnap)
    ec, ew = check.Engine(compact), check.Engine(wsnap)
    out["checks_per_s"] = {
        "compact_hbm": round(timed_hbm(ec, roots, targets)), "writable_hbm": round(timed_hbm(ew, wroots, wtargets)),
        "compact_host": round(timed_host(ec, roots, targets)), "writable_host": round(timed_host(ew, wroots, wtargets))}
    keys = ("plan", "spilled_units", "spilled_requests", "main_ms", "main_bytes", "unit_launches")
    out["run_stats"] = {"compact": {k: ec.last_stats()[k] for k in keys}, "writable": {k: ew.last_stats()[k] for k in keys}}
    log(f"throughput {out['checks_per_s']} stats {out['run_stats']}")
    base_answers = ew.check_ids(wroots, wtargets)
    same0 = int((base_answers == ec.check_ids(roots, targets)).all())
    del ec

    rng = np.random.default_rng(7)
    prng = random.Random(7)
    batches, written = [], []
    for size in [int(x) for x in a.sizes.split(",")]:
        n_ins, n_del = (size + 1) // 2, size // 2
        # inserts into existing groups (a row of a group that has none creates a group: a
        # rebuild), 80% existing users, 20% new ones
        groups = [r[1] for r in membership_rows(w.columns, n_ins, rng)]
        ins = [(1, groups[k], "member",
                f"u{prng.randrange(int(10e6 * f))}" if prng.random() < 0.8 else f"newuser{len(written)}_{k}",
                None, None, None) for k in range(n_ins)]
        dele = membership_rows(w.columns, n_del, rng)
        res = wsnap.write(ins, dele)
        t1 = time.perf_counter()
        if res["applied"]:
            sync_ms, rows = ew.sync()
        else:  # the rebuild path (VersionedEngine's fallback): next version + a new engine
            wsnap = wsnap.apply(ins, dele)
            ew = check.Engine(wsnap)
            sync_ms, rows = 0.0, 0
        entry = {"size": size, "applied": res["applied"], "reason": res["reason"],
                 "write_ms": round(res["seconds"] * 1e3, 3), "sync_ms": round(sync_ms, 3),
                 "total_ms": round(res["seconds"] * 1e3 + (time.perf_counter() - t1) * 1e3, 3),
                 "device_rows": rows, "groups_touched": res["groups_touched"], "new_nodes": res["new_nodes"]}
        if True:
            tuples = [InternalRelationTuple("groups", r[1], "member", SubjectID(r[3])) for r in ins]
            got = ew.check_batch(tuples)
            entry["inserted_allowed"] = f"{int(np.sum(got))}/{len(tuples)}"
        batches.append((ins, dele))
        written += ins + dele
        out.setdefault("writes", []).append(entry)
        log(f"write {entry}")

    # checks after the writes: the writable engine keeps its plan (label: heads rewritten in place)
    st = ew.last_stats()
    out["after_writes"] = {"rows_written": len(written), "plan": st["plan"],
                           "writable_host": round(timed_host(ew, wroots, wtargets)),
                           "writable_hbm": round(timed_hbm(ew, wroots, wtargets)),
                           "label_rewritten": st["label_rewritten"], "label_marked": st["label_marked"],
                           "label_relabels": st["label_relabels"]}
    log(f"after the writes: {out['after_writes']}")
    if a.nest:  # nesting edges between existing groups: changes the interior graph
        gcols = w.columns
        kind, ns = gcols["subject_kind"], gcols["namespace_id"]
        sets = np.flatnonzero((ns == 1) & (kind == 1))
        pick = sets[rng.integers(0, len(sets), size=2 * a.nest)]
        sv = lambda c, i: bytes(gcols[c + "_data"][gcols[c + "_off"][i]:gcols[c + "_off"][i + 1]]).decode()
        # a parent that already nests a group gets another existing nested group (both interior)
        ins = [(1, sv("object", pick[2 * k]), "member", None, 1, sv("ss_object", pick[2 * k + 1]), "member")
               for k in range(a.nest)]
        res = wsnap.write(ins, [])
        t1 = time.perf_counter()
        sync_ms, rows = ew.sync() if res["applied"] else (0.0, 0)
        entry = {"nest_rows": a.nest, "applied": res["applied"], "reason": res["reason"],
                 "write_ms": round(res["seconds"] * 1e3, 3), "sync_ms": round(sync_ms, 3),
                 "total_ms": round(res["seconds"] * 1e3 + (time.perf_counter() - t1) * 1e3, 3)}
        if res["applied"]:
            batches.append((ins, []))
            written += ins
            h = timed_host(ew, wroots, wtargets)
            st = ew.last_stats()
            entry.update(writable_host_after=round(h), plan=st["plan"], label_marked=st["label_marked"],
                         label_relabels=st["label_relabels"], rest_requests=st["rest_requests"])
        out["nest_write"] = entry
        log(f"nesting write {entry}")
        if res["applied"] and a.relabel_permille is not None:
            # a background relabel started by the write: checks while it runs, the swap (at an
            # engine sync once the labels are built), checks after it
            before = st["label_relabels"]
            t_w = time.perf_counter()
            during = round(timed_host(ew, wroots, wtargets))
            swap_sync_ms = None
            while time.perf_counter() - t_w < 120:
                t2 = time.perf_counter()
                ew.sync()
                ew.check_ids(wroots[:1], wtargets[:1])
                dt2 = (time.perf_counter() - t2) * 1e3  # (the swap runs in whichever of the two syncs first)
                if ew.last_stats()["label_relabels"] > before:
                    swap_sync_ms = round(dt2, 3)
                    break
                time.sleep(0.005)
            swap_s = round(time.perf_counter() - t_w, 3)
            after = round(timed_host(ew, wroots, wtargets))
            st = ew.last_stats()
            out["background_relabel"] = {"relabel_permille": a.relabel_permille, "checks_host_during": during,
                                         "swapped_after_s": swap_s, "swap_sync_ms": swap_sync_ms,
                                         "checks_host_after": after, "label_relabels": st["label_relabels"],
                                         "label_marked_after": st["label_marked"], "plan": st["plan"]}
            log(f"background relabel {out['background_relabel']}")

    # the rebuild path on the compact snapshot, and the cross-check
    t0 = time.time()
    cur = compact
    rebuild_s = []
    for ins, dele in batches:  # the compact snapshot through the rebuild path
        t1 = time.time()
        cur = cur.apply(ins, dele)
        rebuild_s.append(round(time.time() - t1, 1))
    out["rebuild_s_per_batch"] = rebuild_s
    log(f"rebuilt in {time.time() - t0:.1f}s: {rebuild_s}")
    er = check.Engine(cur)
    idx = np.random.default_rng(3).permutation(w.n_checks)[:a.sample]
    reqs = [InternalRelationTuple(ns, o, r, SubjectID(s["subject_id"])) for ns, o, r, s in w.requests(idx)]
    reqs += [InternalRelationTuple("groups", r[1], "member", SubjectID(r[3])) for r in written]
    reqs += [InternalRelationTuple("docs", f"d{prng.randrange(int(2e6 * f))}", "viewer", SubjectID(r[3]))
             for r in written]
    got, want = ew.check_batch(reqs), er.check_batch(reqs)
    out["cross_check"] = {"requests": len(reqs), "mismatches": int(np.sum(np.asarray(got) != np.asarray(want))),
                          "against": "engine over the rebuilt snapshot (ketogpu_snapshot_apply per batch)",
                          "before_writes_equal": bool(same0)}
    log(f"cross-check {out['cross_check']}")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
