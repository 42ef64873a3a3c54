"""In-place writes on writable snapshots (R14 at O(delta)).

ketogpu_snapshot_write must leave a writable snapshot equal — by node identity, since ids
differ — to a full reload of the written table: the same expand trees (host rows, order
included), the same resolution, and the same device rows once the free-slot placeholders
are stripped.  Batches the free slots cannot represent must be refused with the snapshot
unchanged, and VersionedEngine must then rebuild.  The GPU tests check answers against
the oracle after every write (internal/persistence/sql/relationtuples.go:128-278)."""
import json
import random

import numpy as np
import pytest

from keto_amd import _lib as L
from keto_amd import expand
from keto_amd import relationtuple as rt
from keto_amd.snapshot import Snapshot
from tests import randgraph
from tests.test_freshness import _expected, _sqlite_key

NODE_NONE = L.NODE_NONE


def _graph(seed, n_rows=400, n_obj=14, n_users=12):
    # no wildcard subject sets and no poisoned pages: the graphs in-place writes serve
    return randgraph.make_graph(seed, n_rows=n_rows, n_obj=n_obj, n_users=n_users, wildcard=False, poison=False)


def _universe(namespaces, rows, extra_users=()):
    objs = {x[1] for x in rows} | {x[5] for x in rows if x[5]}
    rels = {x[2] for x in rows} | {x[6] for x in rows if x[6]}
    sets = sorted((ns, o, r) for ns, _ in namespaces for o in objs for r in rels)
    users = sorted({x[3] for x in rows if x[3] is not None} | set(extra_users))
    return sets, users


def _named(snap, namespaces, sets, users):
    """device rows by node identity: {name: sorted successor names}, {name: sorted predecessor
    names}, and the ids no name resolves to (the placeholders of a writable layout)"""
    inv = {}
    ns0 = namespaces[0][0]
    for ns, o, r in sets:  # as a subject: sets without rows have nodes too
        _, v = snap.resolve(ns0, "o0", "r0", rt.SubjectSet(ns, o, r))
        if v != NODE_NONE:
            inv[v] = ("set", ns, o, r)
    for u in users:
        _, t = snap.resolve(ns0, "o0", "r0", rt.SubjectID(u))
        if t != NODE_NONE:
            inv[t] = ("id", u)
    g = snap.graph()
    unknown = set()
    fwd, rev = {}, {}
    for v in range(g["Nx"]):
        row = g["fint_col"][g["fint_off"][v]:g["fint_off"][v + 1]]
        names = sorted(inv[int(u)] for u in row if int(u) in inv)
        unknown |= {int(u) for u in row if int(u) not in inv}
        if names:
            fwd[inv.get(v, ("?", v))] = names
    for u in range(g["N"]):
        row = g["rev_col"][g["rev_off"][u]:g["rev_off"][u + 1]]
        names = sorted(inv[int(p)] for p in row if int(p) in inv)
        unknown |= {int(p) for p in row if int(p) not in inv}
        if names:
            rev[inv.get(u, ("?", u))] = names
    interior = {inv[v] for v in inv if v < g["Ni"]}
    return fwd, rev, unknown, interior


def _trees(snap, namespaces, sets):
    e = expand.Engine(snap)
    out = {}
    for ns, o, r in sets:
        try:
            out[(ns, o, r)] = e.build_tree_json(rt.SubjectSet(ns, o, r), 3)
        except expand.NotFound:
            out[(ns, o, r)] = "not_found"
    return out


def _writes(seed, namespaces, rows, n_ins=10, n_del=8, new_groups=False):
    """a write batch of mostly representable rows: existing groups gain existing or new
    subject ids and existing subject sets; existing rows are deleted"""
    rng = random.Random(seed)
    groups = sorted({(r[0], r[1], r[2]) for r in rows})
    subj_sets = sorted({(r[4], r[5], r[6]) for r in rows if r[3] is None})
    ins = []
    for _ in range(n_ins):
        ns, o, r = rng.choice(groups)
        x = rng.random()
        if x < 0.45:
            ins.append((ns, o, r, f"u{rng.randrange(16)}", None, None, None))
        elif x < 0.6:
            ins.append((ns, o, r, f"fresh{seed % 97}_{rng.randrange(6)}", None, None, None))
        elif x < 0.8 and subj_sets:
            sns, so, sr = rng.choice(subj_sets)
            ins.append((ns, o, r, None, sns, so, sr))
        else:
            ins.append(rng.choice(rows))  # a duplicate row
        if new_groups and rng.random() < 0.05:
            ins.append((ns, f"brand_new{rng.randrange(3)}", r, "u1", None, None, None))
    dele = [rng.choice(rows) for _ in range(n_del)] + [(groups[0][0], "nothing", "r0", "nobody", None, None, None)]
    return ins, dele


def _assert_same(w, r, namespaces, sets, users):
    """the reverse rows hold every edge (p -> u for expandable p): equal by identity.  The
    forward rows hold the interior successors; node classes of a writable snapshot are fixed
    between rebuilds, so it may keep a node interior that a reload classifies otherwise — only
    one that no longer has rows or is no longer named by any row (no path passes through it)"""
    fw, rw, unk_w, iw = _named(w, namespaces, sets, users)
    fr, rr, unk_r, ir = _named(r, namespaces, sets, users)
    assert rw == rr
    assert not unk_r and len(unk_w) <= 3  # Df, Dbi, Dbo
    preds = {p for ps in rr.values() for p in ps}  # nodes with rows
    # interior only in the writable one: it lost its rows or every row naming it
    assert ir <= iw and all(x not in preds or x not in rr for x in iw - ir)
    for f, interior in ((fw, iw), (fr, ir)):
        succ = {}
        for u, ps in rr.items():
            for p in ps:
                if u in interior:
                    succ.setdefault(p, []).append(u)
        assert f == {p: sorted(us) for p, us in succ.items()}
    assert _trees(w, namespaces, sets) == _trees(r, namespaces, sets)
    assert w.stats()["num_rows"] == r.stats()["num_rows"]


def _all_users(seed, steps):
    return [f"u{k}" for k in range(16)] + [f"fresh{(seed * 10 + s) % 97}_{k}" for s in range(steps) for k in range(6)]


@pytest.mark.parametrize("seed,order", [(301, "sqlite"), (302, "postgres"), (303, "sqlite")])
def test_in_place_writes_equal_a_reload(seed, order):
    namespaces, rows = _graph(seed)
    w = Snapshot.from_rows(namespaces, rows, sort=True, order=order, writable=True)
    cur = sorted(rows, key=_sqlite_key)
    applied = 0
    for step in range(6):
        ins, dele = _writes(seed * 10 + step, namespaces, cur)
        res = w.write(ins, dele)
        if res["applied"]:
            applied += 1
            assert res["version"] == w.version()
        else:
            w = w.apply(ins, dele)  # the rebuild keeps the layout writable
        # the reload: the rows, inserts after equal rows (stable sort), deletes removed
        cur = _expected(cur, ins, dele)
        want = Snapshot.from_rows(namespaces, cur, sort=True, order=order)
        sets, users = _universe(namespaces, cur, extra_users=_all_users(seed, step + 1))
        _assert_same(w, want, namespaces, sets, users)
    assert applied >= 4  # most batches are representable


def test_refusals_leave_the_snapshot_unchanged():
    namespaces, rows = _graph(311, n_rows=200)
    w = Snapshot.from_rows(namespaces, rows, sort=True, writable=True)
    sets, users = _universe(namespaces, rows, extra_users=["zz"])
    before = _named(w, namespaces, sets, users), _trees(w, namespaces, sets)
    g = sorted({(r[0], r[1], r[2]) for r in rows})[0]
    cases = [
        ([(g[0], "brand_new", g[2], "u1", None, None, None)], "class"),   # a new group
        ([(99, g[1], g[2], "u1", None, None, None)], "poison"),           # unconfigured namespace id
        ([(g[0], g[1], g[2], None, 99, "o1", "r1")], "poison"),           # ... in the subject set
        ([(g[0], g[1], g[2], None, g[0], "", "r1")], "wildcard"),         # an R5 wildcard subject set
    ]
    for ins, reason in cases:
        res = w.write(ins + [(g[0], g[1], g[2], "ok_user", None, None, None)], [])
        assert not res["applied"] and res["reason"] == reason, (ins, res)
    assert (_named(w, namespaces, sets, users), _trees(w, namespaces, sets)) == before
    assert w.version() == 0
    # a full row: one group gains more new subjects than its free slots and reserved ids hold
    many = [(g[0], g[1], g[2], f"flood{k}", None, None, None) for k in range(5000)]
    res = w.write(many, [])
    assert not res["applied"] and res["reason"] in ("reserve", "full")
    assert (_named(w, namespaces, sets, users), _trees(w, namespaces, sets)) == before
    # a snapshot that is not writable, and one with wildcard subject sets
    assert Snapshot.from_rows(namespaces, rows, sort=True).write(many[:1], [])["reason"] == "not_writable"
    nsw, roww = randgraph.make_graph(312, n_rows=200, wildcard=True)
    if any(r[5] == "" or r[6] == "" for r in roww):
        ww = Snapshot.from_rows(nsw, roww, sort=True, writable=True)
        assert ww.write([roww[0]], [])["reason"] == "wildcard"


def test_shared_string_keys_are_refused():
    """R4: a new subject id whose Subject.String() equals an existing subject set's"""
    ns = [("n0", 1)]
    rows = [(1, "o1", "r1", None, 1, "o2", "r2"), (1, "o2", "r2", "u1", None, None, None)]
    w = Snapshot.from_rows(ns, rows, sort=True, writable=True)
    res = w.write([(1, "o1", "r1", "n0:o2#r2", None, None, None)], [])
    assert not res["applied"] and res["reason"] == "ambiguous"
    assert w.write([(1, "o1", "r1", "plain", None, None, None)], [])["applied"]


def test_written_snapshot_round_trips_through_a_file(tmp_path):
    namespaces, rows = _graph(321)
    w = Snapshot.from_rows(namespaces, rows, sort=True, writable=True)
    ins, dele = _writes(3210, namespaces, rows)
    assert w.write(ins, dele)["applied"]
    w.save(tmp_path / "w.snap")
    back = Snapshot.load(tmp_path / "w.snap")
    ga, gb = w.graph(), back.graph()
    for k in ("fint_off", "fint_col", "rev_off", "rev_col"):
        np.testing.assert_array_equal(ga[k], gb[k])
    cur = _expected(sorted(rows, key=_sqlite_key), ins, dele)
    ins2, dele2 = _writes(3211, namespaces, cur)
    a, b = w.write(ins2, dele2), back.write(ins2, dele2)
    assert a["applied"] == b["applied"]
    sets, users = _universe(namespaces, cur, extra_users=[f"fresh{3211 % 97}_{k}" for k in range(6)] +
                            [f"u{k}" for k in range(16)])
    assert _named(w, namespaces, sets, users) == _named(back, namespaces, sets, users)


def _tuple(r, id2name):
    s = rt.SubjectID(r[3]) if r[3] is not None else rt.SubjectSet(id2name[r[4]], r[5], r[6])
    return rt.InternalRelationTuple(id2name[r[0]], r[1], r[2], s)


@pytest.mark.gpu
@pytest.mark.parametrize("plan", ["label", "label-marks", "label-relabel", "label-relabel-sync", "lite"])
def test_versioned_engine_writes_in_place_and_reads_them(plan, monkeypatch):
    """read-your-writes against the oracle after every batch; most batches in place, a
    batch with a new group through the rebuild.  Plan label keeps its labels exact in place
    (label_update: changed rows' heads rewritten, roots above a changed nesting edge sent to
    the second stage), relabelling past the default share of marked heads, never
    (label-marks) or at every marked head (label-relabel: in the background, swapped in at a
    later sync; label-relabel-sync: inline); plan lite for comparison"""
    from keto_amd.freshness import VersionedEngine
    if L.lib().ketogpu_device_count() < 1:
        pytest.fail("no HIP device visible")
    if plan == "lite":
        monkeypatch.setenv("KETOGPU_NO_LABEL", "1")
    elif plan == "label-marks":
        monkeypatch.setenv("KETOGPU_LABEL_RELABEL_PERMILLE", "1000")
    elif plan.startswith("label-relabel"):
        monkeypatch.setenv("KETOGPU_LABEL_RELABEL_PERMILLE", "0")
        if plan == "label-relabel-sync":
            monkeypatch.setenv("KETOGPU_LABEL_RELABEL_SYNC", "1")
    namespaces, rows = _graph(331, n_rows=700, n_obj=25, n_users=30)
    ve = VersionedEngine(Snapshot.from_rows(namespaces, rows, sort=True, writable=True))
    id2name = {i: n for n, i in namespaces}
    cur = sorted(rows, key=_sqlite_key)
    paths = []
    marks = relabels = 0
    for step in range(8):
        ins, dele = _writes(400 + step, namespaces, cur, new_groups=(step == 5))
        ve.transact(insert=[_tuple(r, id2name) for r in ins], delete=[_tuple(d, id2name) for d in dele])
        paths.append(ve.last_write["path"])
        cur = _expected(cur, ins, dele)
        eng = ve._state[1]
        assert eng.check_graph() == 0, (step, paths, eng.check_graph_first, eng.last_stats()["plan"])
        reqs = randgraph.make_requests(500 + step, namespaces, cur, n=500, wildcard=False)
        want = randgraph.oracle_store(namespaces, cur).check_batch(reqs)
        tuples = [rt.InternalRelationTuple(ns, o, r, rt.subject_from_dict(s)) for ns, o, r, s in reqs]
        got = ve.check_many(tuples)
        if got != [bool(x) for x in want]:  # diagnose: a fresh writable / compact engine on the same rows
            from keto_amd import check
            fresh_w = check.Engine(Snapshot.from_rows(namespaces, cur, sort=True, writable=True)).check_many(tuples)
            fresh_c = check.Engine(Snapshot.from_rows(namespaces, cur, sort=True)).check_many(tuples)
            bad = [i for i in range(len(want)) if got[i] != bool(want[i])]
            pytest.fail(f"step {step} paths {paths}: {len(bad)} mismatches (e.g. {[reqs[i] for i in bad[:3]]}); "
                        f"fresh writable engine {sum(a != bool(b) for a, b in zip(fresh_w, want))}, "
                        f"fresh compact engine {sum(a != bool(b) for a, b in zip(fresh_c, want))}")
        assert list(ve._state[1].check_batch(tuples)) == [bool(x) for x in want], step  # the id path
        st = eng.last_stats()
        assert (st["plan"] == 7) == (plan != "lite"), (step, st["plan"])
        if plan != "lite" and ve.last_write["path"] == "in_place":
            marks += st["label_marked"] > 0
            relabels = max(relabels, st["label_relabels"])
        orc = randgraph.oracle_store(namespaces, cur)
        known = {n for n, _ in namespaces}
        for ns, o, r, _ in [q for q in reqs if q[0] in known][:40]:
            got = json.loads(ve._state[2].build_tree_json(rt.SubjectSet(ns, o, r), 3))
            want_tree = orc.expand({"subject_set": {"namespace": ns, "object": o, "relation": r}}, 3)
            assert got == want_tree, (step, ns, o, r)
    assert paths.count("in_place") >= 5 and "rebuild" in paths, paths
    if plan == "label-marks":
        assert marks > 0 and relabels == 0  # nesting edges changed: roots marked, never relabelled
    if plan == "label-relabel-sync":
        assert relabels > 0


@pytest.mark.gpu
def test_checks_during_a_background_relabel(monkeypatch):
    """a write that marks roots starts a background relabel (KETOGPU_LABEL_RELABEL_PERMILLE=0:
    at the first mark) and returns; checks run while the labels are built (marked roots on
    the second stage) and after the swap (the new heads, every row changed since the copy
    re-applied), each batch equal to the oracle, until the engine reports the relabel"""
    import time as _time
    from keto_amd.freshness import VersionedEngine
    monkeypatch.setenv("KETOGPU_LABEL_RELABEL_PERMILLE", "0")
    namespaces, rows = _graph(337, n_rows=700, n_obj=25, n_users=30)
    ve = VersionedEngine(Snapshot.from_rows(namespaces, rows, sort=True, writable=True))
    id2name = {i: n for n, i in namespaces}
    cur = sorted(rows, key=_sqlite_key)
    swapped = 0
    for step in range(4):
        ins, dele = _writes(460 + step, namespaces, cur)
        ve.transact(insert=[_tuple(r, id2name) for r in ins], delete=[_tuple(d, id2name) for d in dele])
        cur = _expected(cur, ins, dele)
        reqs = randgraph.make_requests(560 + step, namespaces, cur, n=400, wildcard=False)
        want = [bool(x) for x in randgraph.oracle_store(namespaces, cur).check_batch(reqs)]
        tuples = [rt.InternalRelationTuple(ns, o, r, rt.subject_from_dict(s)) for ns, o, r, s in reqs]
        eng = ve._state[1]
        before = eng.last_stats()["label_relabels"] if step else 0
        for k in range(200):  # checks while the relabel runs, then after its swap
            assert ve.check_many(tuples) == want, (step, k)
            st = eng.last_stats()
            assert st["plan"] == 7
            if st["label_relabels"] > before:
                swapped += 1
                break
            _time.sleep(0.01)
        assert ve.check_many(tuples) == want
    assert swapped > 0


def test_hub_fanout_is_refused_past_the_budget(monkeypatch):
    """a nested-group insert into a group that many documents reference changes
    the group's interior-successor count, which every predecessor's forward records carry;
    past KETOGPU_WRITE_FANOUT_MAX re-uploaded rows the write is refused (the engine
    rebuilds instead) and the snapshot is unchanged"""
    ns = [("g", 1), ("d", 2)]
    rows = [(1, "hub", "member", None, 1, "s0", "member"), (1, "s0", "member", "u0", None, None, None),
            (1, "s0", "member", None, 1, "s1", "member"),  # s1 is interior already
            (1, "s1", "member", "u1", None, None, None), (1, "s1", "member", None, 1, "s2", "member"),
            (1, "s2", "member", "u2", None, None, None)]
    rows += [(2, f"doc{k}", "viewer", None, 1, "hub", "member") for k in range(40)]
    ins = [(1, "hub", "member", None, 1, "s1", "member")]  # hub's interior successors 1 -> 2
    w = Snapshot.from_rows(ns, rows, sort=True, writable=True)
    monkeypatch.setenv("KETOGPU_WRITE_FANOUT_MAX", "10")
    res = w.write(ins, [])
    assert not res["applied"] and res["reason"] == "fanout"
    assert w.version() == 0
    monkeypatch.setenv("KETOGPU_WRITE_FANOUT_MAX", "1000")
    res = w.write(ins, [])
    assert res["applied"] and res["device_rows"] >= 40
