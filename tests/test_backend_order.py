"""Backend-faithful row order.  The ORDER BY of
internal/persistence/sql/relationtuples.go:215 is executed by the backend; Postgres
sorts NULLs last, so a group's subject-id rows precede its subject-set rows there, and
expand child order (R9/R10) follows.  These tests pin the Postgres order (NULLS LAST, "C"
collation) three ways: the oracle's restatement against real SQL (SQLite executing the
same ORDER BY with NULLS LAST), the snapshot built from rows in that order, and the
write path (ketogpu_snapshot_apply) merging in it.  Locale collations stay unpinned."""
import random

import pytest

from keto_amd import expand, persistence
from keto_amd import relationtuple as rt
from keto_amd.snapshot import Snapshot
from oracle import oracle as O
from tests import randgraph
from tests.sqlite_reference import SqliteReference
from tests.test_oracle import as_tuple_subject


def _trees(snap_or_store, namespaces, objs, rels=("r0", "r1", ""), depth=3):
    out = []
    for ns, _ in namespaces:
        for o in objs:
            for rel in rels:
                s = {"subject_set": {"namespace": ns, "object": o, "relation": rel}}
                try:
                    if isinstance(snap_or_store, expand.Engine):
                        t = snap_or_store.BuildTree(rt.subject_from_dict(s), depth)
                        out.append(t.to_node() if t else None)
                    else:
                        out.append(snap_or_store.expand(s, depth))
                except (expand.NotFound, O.OracleError):
                    out.append("not_found")
    return out


@pytest.mark.parametrize("seed,page_size", [(301, 100), (302, 3), (303, 1)])
def test_postgres_order_oracle_matches_sql(seed, page_size):
    namespaces, rows = randgraph.make_graph(seed, n_rows=160, poison=True, empty_ns=True)
    store = persistence.TupleStore(namespaces, page_size=page_size, order="postgres")
    for i, (ns, o, r, sid, sns, so, sr) in enumerate(rows):
        store.insert_raw(ns, o, r, sid, sns, so, sr, commit_time=i)
    ref = SqliteReference(store)
    orc = randgraph.oracle_store(namespaces, rows, page_size, order="postgres")
    for ns in [n for n, _ in namespaces] + ["unknown"]:
        for o in ["", "o1", "o2"]:
            for r in ["", "r0"]:
                for page in (1, 2):
                    try:
                        want = ref.get_relation_tuples(ns, o, r, page)
                    except Exception:
                        want = "not_found"
                    try:
                        got, nxt = orc.get_page(ns, o, r, page)
                        got = ([as_tuple_subject(x) for x in got], nxt)
                    except O.OracleError:
                        got = "not_found"
                    assert got == want, (ns, o, r, page)
    for (ns, o, r, subj) in randgraph.make_requests(seed, namespaces, rows, n=40):
        for depth in (1, 2, 5):
            s = {"subject_set": {"namespace": ns, "object": o, "relation": r}}
            try:
                want = ref.expand(as_tuple_subject(s), depth)
            except Exception:
                want = "not_found"
            try:
                got = orc.expand(s, depth)
            except O.OracleError:
                got = "not_found"
            assert got == want, (s, depth)


@pytest.mark.parametrize("seed,page_size", [(311, 100), (312, 2)])
def test_postgres_order_snapshot_expand(seed, page_size):
    namespaces, rows = randgraph.make_graph(seed, n_rows=300, poison=True, empty_ns=True)
    orc = randgraph.oracle_store(namespaces, rows, page_size, order="postgres")
    objs = sorted({r[1] for r in rows})[:10]
    want = _trees(orc, namespaces, objs)
    # rows read in Postgres order (the loader keeps them), and unordered rows sorted by it
    pg = Snapshot.from_rows(namespaces, randgraph.backend_sorted(rows, "postgres"), page_size=page_size, sort=False,
                            order="postgres")
    assert _trees(expand.Engine(pg), namespaces, objs) == want
    srt = Snapshot.from_rows(namespaces, rows, page_size=page_size, sort=True, order="postgres")
    assert _trees(expand.Engine(srt), namespaces, objs) == want
    # the SQLite-ordered snapshot differs where a group mixes subject ids and subject sets
    lite = Snapshot.from_rows(namespaces, rows, page_size=page_size, sort=True)
    assert _trees(expand.Engine(lite), namespaces, objs) == _trees(
        randgraph.oracle_store(namespaces, rows, page_size), namespaces, objs)
    assert _trees(expand.Engine(lite), namespaces, objs) != want
    # the store loader (one ordered read, NULLS LAST) gives the same snapshot as the sorted build
    store = persistence.TupleStore(namespaces, page_size=page_size, order="postgres")
    for i, r in enumerate(rows):
        store.insert_raw(*r, commit_time=i)
    assert _trees(expand.Engine(Snapshot.from_store(store)), namespaces, objs) == want


def test_postgres_order_apply_and_persist(tmp_path):
    namespaces, rows = randgraph.make_graph(321, n_rows=400, n_obj=15, poison=True, empty_ns=True)
    base = Snapshot.from_rows(namespaces, rows, sort=True, order="postgres")
    rng = random.Random(5)
    ins = [rng.choice(rows) for _ in range(20)]
    ins += [(1, f"o{rng.randrange(15)}", "r0", f"new{i}", None, None, None) for i in range(15)]
    ins += [(1, f"o{rng.randrange(15)}", "r1", None, 2, "o3", "r0") for _ in range(15)]
    dele = [rng.choice(rows) for _ in range(25)]
    got = base.apply(ins, dele)
    keys = set(dele)
    want_rows = [r for r in randgraph.backend_sorted(rows, "postgres") + ins if r not in keys]
    want = Snapshot.from_rows(namespaces, want_rows, sort=True, order="postgres")
    objs = sorted({r[1] for r in want_rows})
    assert _trees(expand.Engine(got), namespaces, objs) == _trees(expand.Engine(want), namespaces, objs)
    assert _trees(expand.Engine(got), namespaces, objs) == _trees(
        randgraph.oracle_store(namespaces, want_rows, order="postgres"), namespaces, objs)
    # the order survives save/load: a later write merges the Postgres way
    got.save(tmp_path / "pg.snap")
    back = Snapshot.load(tmp_path / "pg.snap", namespaces)
    more = [(1, "o1", "r0", "zz", None, None, None), (1, "o1", "r0", None, 1, "o2", "r2")]
    a, b = back.apply(more), got.apply(more)
    assert _trees(expand.Engine(a), namespaces, ["o1"]) == _trees(expand.Engine(b), namespaces, ["o1"])
    t = expand.Engine(a).BuildTree(rt.SubjectSet(namespaces[0][0], "o1", "r0"), 2)
    kinds = [isinstance(c.subject, rt.SubjectSet) for c in t.children]
    assert kinds == sorted(kinds)  # subject ids (False) before subject sets (True)
