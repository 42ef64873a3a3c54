"""Write-path freshness (R14): ketogpu_snapshot_apply must produce
exactly the snapshot a full reload of the written table would (same ORDER BY with
commit_time last, delete-all-duplicates), and VersionedEngine must answer with every
acknowledged write applied (read-your-writes, internal/persistence/sql/
relationtuples.go:128-278)."""
import random

import numpy as np
import pytest

from keto_amd import _lib as L
from keto_amd import expand
from keto_amd import relationtuple as rt
from keto_amd.snapshot import Snapshot
from tests import randgraph


def _sqlite_key(row):
    # ORDER BY of relationtuples.go:215 with SQLite NULL-first / BINARY semantics (commit_time = position)
    ns, o, r, sid, sns, so, sr = row
    b = lambda s: (s or "").encode()
    return (ns, b(o), b(r), sid is not None, b(sid), sns if sns is not None else -1, b(so), b(sr))


def _write_batch(seed, namespaces, rows):
    rng = random.Random(seed)
    ids = [i for _, i in namespaces] + [99]  # 99: an unconfigured id poisons pages
    ins = []
    for _ in range(60):
        base = rng.choice(rows)
        if rng.random() < 0.3:
            ins.append(base)  # a duplicate
        elif rng.random() < 0.5:
            ins.append((rng.choice(ids), base[1], rng.choice(["r0", "r1", "new"]), f"fresh{rng.randrange(9)}",
                        None, None, None))
        else:
            ins.append((rng.choice(ids), f"o{rng.randrange(14)}", base[2], None, rng.choice(ids),
                        rng.choice([base[1], "o3", "", "zz"]), rng.choice(["r0", "r2", ""])))
    dele = [rng.choice(rows) for _ in range(40)] + [(ids[0], "nothing", "r0", "nobody", None, None, None)]
    return ins, dele


def _expected(rows, ins, dele):
    ordered = sorted(rows, key=_sqlite_key)  # the base as the loader read it
    keys = {(d[0], d[1], d[2], d[3], d[4], d[5], d[6]) for d in dele}
    return [r for r in ordered + list(ins) if tuple(r) not in keys]


def _same(a, b):
    sa, sb = a.stats(), b.stats()
    sa.pop("build_seconds"), sb.pop("build_seconds")
    assert sa == sb
    ga, gb = a.graph(), b.graph()
    for k in ("fint_off", "fint_col", "rev_off", "rev_col"):
        np.testing.assert_array_equal(ga[k], gb[k])


@pytest.mark.parametrize("seed,page_size,collide", [(101, 100, False), (102, 3, False), (103, 2, True)])
def test_apply_equals_full_reload(seed, page_size, collide):
    namespaces, rows = randgraph.make_graph(seed, n_rows=500, n_obj=15, poison=True, collide=collide, empty_ns=True)
    base = Snapshot.from_rows(namespaces, rows, page_size=page_size, sort=True)
    ins, dele = _write_batch(seed, namespaces, rows)
    got = base.apply(ins, dele)
    want_rows = _expected(rows, ins, dele)
    want = Snapshot.from_rows(namespaces, want_rows, page_size=page_size, sort=True)
    _same(got, want)
    assert got.stats()["num_rows"] == len(want_rows)
    # expand trees (order-sensitive) and the page-poisoned errors agree
    e_got, e_want = expand.Engine(got), expand.Engine(want)
    objs = sorted({r[1] for r in want_rows})[:12]
    for ns, _ in namespaces:
        for o in objs:
            for rel in ("r0", "r1", ""):
                s = rt.SubjectSet(ns, o, rel)
                res = []
                for e in (e_got, e_want):
                    try:
                        res.append(e.build_tree_json(s, 3))
                    except expand.NotFound:
                        res.append("not_found")
                assert res[0] == res[1], (ns, o, rel)
    # the base is unchanged and a chain of versions equals one reload
    _same(base, Snapshot.from_rows(namespaces, rows, page_size=page_size, sort=True))
    ins2, dele2 = _write_batch(seed + 50, namespaces, want_rows)
    _same(got.apply(ins2, dele2),
          Snapshot.from_rows(namespaces, _expected(want_rows, ins2, dele2), page_size=page_size, sort=True))


def test_apply_delete_everything_and_empty_batches():
    rows = [(1, "o", "r", "u", None, None, None), (1, "o", "r", "u", None, None, None)]
    base = Snapshot.from_rows([("n", 1)], rows)
    _same(base.apply(), base)
    empty = base.apply(delete_rows=[rows[0]])  # both duplicates go
    assert empty.stats()["num_rows"] == 0


@pytest.mark.parametrize("seed", [121, 122])
def test_namespace_reload_equals_a_load_under_the_new_config(seed):
    """ketogpu_snapshot_set_namespaces: removing a namespace poisons the pages of its rows
    (R7), renaming changes resolution, re-adding heals; each equals a fresh load of the same
    rows under that configuration (expand trees, errors and the device graph)"""
    namespaces, rows = randgraph.make_graph(seed, n_rows=500, n_obj=15, poison=True)
    base = Snapshot.from_rows(namespaces, rows, page_size=4, sort=True)
    configs = [namespaces[:-1],                                      # a namespace removed
               [(n + "x", i) for n, i in namespaces],                # renamed
               namespaces + [("n9", 98)],                            # the poisoning id 98 configured
               namespaces]                                           # back to the original
    cur = base
    for cfg in configs:
        cur = cur.set_namespaces(cfg)
        want = Snapshot.from_rows(cfg, rows, page_size=4, sort=True)
        _same(cur, want)
        e_got, e_want = expand.Engine(cur), expand.Engine(want)
        for ns, _ in cfg:
            for o in sorted({r[1] for r in rows})[:8]:
                for rel in ("r0", "r1"):
                    res = []
                    for e in (e_got, e_want):
                        try:
                            res.append(e.build_tree_json(rt.SubjectSet(ns, o, rel), 3))
                        except expand.NotFound:
                            res.append("not_found")
                    assert res[0] == res[1], (cfg, ns, o, rel)
    with pytest.raises(L.KetoError):
        base.set_namespaces([("a", 1), ("a", 2)])  # duplicate names are refused


@pytest.mark.gpu
def test_versioned_engine_namespace_reload():
    from keto_amd.freshness import VersionedEngine
    if L.lib().ketogpu_device_count() < 1:
        pytest.fail("no HIP device visible")
    namespaces, rows = randgraph.make_graph(131, n_rows=600, n_obj=25, n_users=30, poison=True)
    ve = VersionedEngine(Snapshot.from_rows(namespaces, rows, sort=True))
    for cfg in (namespaces[:-1], namespaces[1:] + [("extra", 98)], namespaces):
        ve.reload_namespaces(cfg)
        reqs = randgraph.make_requests(140, cfg, rows, n=400)
        want = randgraph.oracle_store(cfg, rows).check_batch(reqs)
        got = ve.check_many([rt.InternalRelationTuple(ns, o, r, rt.subject_from_dict(s)) for ns, o, r, s in reqs])
        assert got == [bool(x) for x in want], cfg


@pytest.mark.gpu
def test_versioned_engine_reads_its_writes():
    from keto_amd.freshness import VersionedEngine
    if L.lib().ketogpu_device_count() < 1:
        pytest.fail("no HIP device visible")
    namespaces, rows = randgraph.make_graph(111, n_rows=600, n_obj=25, n_users=30, poison=True)
    base = Snapshot.from_rows(namespaces, rows, sort=True)
    ve = VersionedEngine(base)
    id2name = {i: n for n, i in namespaces}
    cur = sorted(rows, key=_sqlite_key)
    for step in range(4):
        ins, dele = _write_batch(200 + step, namespaces, cur)
        ins = [r for r in ins if r[0] in id2name and (r[4] is None or r[4] in id2name)]  # names must resolve
        dele = [d for d in dele if d[0] in id2name and (d[4] is None or d[4] in id2name)]

        def tup(r):
            s = rt.SubjectID(r[3]) if r[3] is not None else rt.SubjectSet(id2name[r[4]], r[5], r[6])
            return rt.InternalRelationTuple(id2name[r[0]], r[1], r[2], s)
        v = ve.transact(insert=[tup(r) for r in ins], delete=[tup(d) for d in dele])
        assert v == step + 1
        cur = _expected(cur, ins, dele)
        reqs = randgraph.make_requests(300 + step, namespaces, cur, n=400)
        want = randgraph.oracle_store(namespaces, cur).check_batch(reqs)
        got = ve.check_many([rt.InternalRelationTuple(ns, o, r, rt.subject_from_dict(s)) for ns, o, r, s in reqs])
        assert got == [bool(x) for x in want], step


def test_failed_sync_after_in_place_write_still_commits(monkeypatch):
    """an in-place write is in the shared snapshot before the engine's device
    sync; a sync that raises must not turn into a failed transaction.  The engine is
    rebuilt over the written snapshot (version bumped, path reported); when the rebuild
    fails as well, the transaction still returns its version and reads raise instead of
    answering without the committed write."""
    from keto_amd import freshness

    built = []

    class StubEngine:  # the device engine's interface, on CPU
        fail_sync = True
        fail_new = False

        def __init__(self, snapshot, device=0, **kw):
            if StubEngine.fail_new:
                raise L.KetoError(L.EDEVICE, "stub: no device")
            self.snapshot = snapshot
            built.append(snapshot)

        def sync(self):
            if StubEngine.fail_sync:
                raise L.KetoError(L.EDEVICE, "stub: sync failed")
            return 0.0, 0

        def check_many(self, tuples):
            return [False] * len(tuples)

    monkeypatch.setattr(freshness.check, "Engine", StubEngine)
    rows = [(1, "g", "member", "u1", None, None, None), (1, "d", "viewer", None, 1, "g", "member")]
    ve = freshness.VersionedEngine(Snapshot.from_rows([("n", 1)], rows, writable=True))
    t = rt.InternalRelationTuple("n", "g", "member", rt.SubjectID("u2"))
    assert ve.transact(insert=[t]) == 1
    assert ve.last_write["path"] == "in_place+rebuild" and "sync failed" in ve.last_write["sync_error"]
    assert len(built) == 2 and built[-1].stats()["num_rows"] == 3  # rebuilt over the written rows
    StubEngine.fail_new = True
    t3 = rt.InternalRelationTuple("n", "g", "member", rt.SubjectID("u3"))
    # the newest engine syncs fine; make the sync fail again and the rebuild fail too: the
    # transaction is committed (its version is returned), the engine FAILED
    assert ve.transact(insert=[t3]) == 2 and ve.version == 2
    assert ve.last_write["path"] == "in_place+failed" and "write committed" in ve.last_write["engine_error"]
    assert ve.snapshot.stats()["num_rows"] == 4  # the write is committed in the snapshot
    with pytest.raises(L.KetoError, match="no engine holds"):
        ve.check_many([t3])
