"""GPU parity: the MI355X engine (libketogpu.so, device_engine.hip) against the CPU
oracle (reference DFS restated) and the golden reference assertions.  Bit-exact:
every request's allowed bit must equal the oracle's."""
import os

import numpy as np
import pytest

from keto_amd import _lib as L
from keto_amd import check, persistence
from keto_amd import relationtuple as rt
from keto_amd.snapshot import Snapshot
from tests import randgraph

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if L.lib().ketogpu_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")


def tuples_of(reqs):
    return [rt.InternalRelationTuple(ns, o, r, rt.subject_from_dict(s)) for ns, o, r, s in reqs]


def test_golden_checks_on_gpu(golden_cases):
    n = 0
    for c in golden_cases:
        ns = [(x["name"], x["id"]) for x in c["namespaces"]]
        store = persistence.TupleStore(ns, page_size=c["page_size"])
        for t in c["tuples"]:
            store.insert(rt.InternalRelationTuple.from_dict(t))
        eng = check.Engine(Snapshot.from_store(store))
        for q in c["checks"]:
            got = eng.SubjectIsAllowed(rt.InternalRelationTuple.from_dict(q))
            assert got == q["expected"], (c["name"], q)
            n += 1
        eng.close()
    assert n >= 30


def test_nil_subject_is_bad_request():
    eng = check.Engine(Snapshot.from_rows([("n", 1)], [(1, "o", "r", "u", None, None, None)]))
    with pytest.raises(rt.NilSubject):
        eng.SubjectIsAllowed(rt.InternalRelationTuple("n", "o", "r", None))


@pytest.fixture(params=["bidi", "bidi-wide", "v2", "lite", "lite-shift", "lite32", "core", "core-small", "core-none",
                        "label", "label-small", "label-rest"])
def unit_plan(request, monkeypatch):
    """first LDS pass of engines created while active: the default bidirectional units
    (one-wave, 512-slot tables), bidi with the wide 2048-slot table, forward-only unit2, or
    plan lite (per-unit direction) — also with every row begin carried past 2^32 through
    its 64-bit path (KETOGPU_TEST_BEGIN_SHIFT) — lite with 32-request units, and plan core
    (lite over its own record arrays with closure rows, core_index.hpp) with the default
    caps, with caps of 3 (most closures dropped, mixed closure and one-hop rows) and with
    no closure rows at all; plan label (2-hop labels) with the chosen heads, with 8-word heads
    (most lists in the overflow region) and with 40% of the S heads marked unlabelled (the
    second stage, plan lite over the listed requests)"""
    if request.param == "v2":
        monkeypatch.setenv("KETOGPU_UNITS", "v2")
    elif request.param == "lite32":
        monkeypatch.setenv("KETOGPU_UNITS", "lite32")
    elif request.param.startswith("label"):  # plan label (requests without labels: plan lite)
        monkeypatch.setenv("KETOGPU_UNITS", "label")
        if request.param == "label-small":
            monkeypatch.setenv("KETOGPU_LABEL_HEADS", "8,8")
        elif request.param == "label-rest":
            monkeypatch.setenv("KETOGPU_LABEL_REST_PERMILLE", "400")
    elif request.param.startswith("core"):
        monkeypatch.setenv("KETOGPU_UNITS", "core")
        if request.param != "core":
            monkeypatch.setenv("KETOGPU_CLOSURE", "3,3" if request.param == "core-small" else "0,0")
    elif request.param.startswith("lite"):
        monkeypatch.setenv("KETOGPU_UNITS", "lite")
        if request.param == "lite-shift":
            monkeypatch.setenv("KETOGPU_TEST_BEGIN_SHIFT", str(3 << 32))
    else:
        monkeypatch.setenv("KETOGPU_UNITS", "bidi")
    if request.param == "bidi-wide":
        monkeypatch.setenv("KETOGPU_BIDI", "11,256,384,6")
    return request.param


@pytest.mark.parametrize("seed,page_size,poison,collide,empty_ns,words", [
    (31, 100, False, False, False, 0), (32, 3, True, False, True, 0), (33, 2, True, True, False, 0),
    (34, 1, False, True, True, 0), (35, 100, False, False, False, 1), (36, 5, True, True, True, 2)])
def test_random_tables_match_oracle(seed, page_size, poison, collide, empty_ns, words, unit_plan):
    namespaces, rows = randgraph.make_graph(seed, n_rows=600, n_obj=30, n_users=40, poison=poison, collide=collide,
                                            empty_ns=empty_ns)
    snap = Snapshot.from_rows(namespaces, rows, page_size=page_size, sort=True)
    eng = check.Engine(snap, max_words_per_round=words)
    orc = randgraph.oracle_store(namespaces, rows, page_size)
    reqs = randgraph.make_requests(seed, namespaces, rows, n=1000)
    got = eng.check_many(tuples_of(reqs))
    want = orc.check_batch(reqs)
    bad = [(reqs[i], got[i], bool(want[i])) for i in range(len(reqs)) if got[i] != bool(want[i])]
    assert not bad, bad[:5]
    assert any(want) and not all(want)


@pytest.mark.parametrize("heads,permille", [("0,0", 0), ("8,8", 0), ("16,8", 0), ("32,32", 0), ("8,16", 250)])
def test_label_heads_match_oracle(heads, permille, monkeypatch):
    """plan label over lists of up to hundreds of entries (the family graph's wide closures):
    every head size pair (8-word heads: most lists in the overflow region), with a share of
    the S heads marked unlabelled (the second stage), on device, HBM-resident and pinned
    host batches"""
    monkeypatch.setenv("KETOGPU_UNITS", "label")
    monkeypatch.setenv("KETOGPU_LABEL_HEADS", heads)
    monkeypatch.setenv("KETOGPU_LABEL_REST_PERMILLE", str(permille))
    namespaces, rows, reqs = randgraph.make_family_graph(92)
    snap = Snapshot.from_rows(namespaces, rows, sort=True)
    want = randgraph.oracle_store(namespaces, rows).check_batch(reqs)
    eng = check.Engine(snap)
    assert eng.check_many(tuples_of(reqs)) == [bool(x) for x in want]
    st = eng.last_stats()
    assert st["plan"] == 7 and st["label_on"] == 1
    if heads != "0,0":
        assert f'{st["label_s_head"]},{st["label_p_head"]}' == heads
    roots, targets = snap.resolve_many([(ns, o, r, rt.subject_from_dict(x)) for ns, o, r, x in reqs])
    q = eng.upload(roots, targets)  # HBM-resident
    q.run()
    np.testing.assert_array_equal(q.download(), want)
    assert (eng.last_stats()["rest_requests"] > 0) == (permille > 0)
    pr, pt = check.pinned(roots), check.pinned(targets)  # pinned host requests read in place
    out = check.PinnedBuffer((len(roots) + 63) // 64, np.uint64)
    eng.check_ids_raw(pr.array.ctypes.data, pt.array.ctypes.data, len(roots), out.array.ctypes.data)
    np.testing.assert_array_equal(check.unpack_bits(out.array.copy(), len(roots)), want)


@pytest.mark.parametrize("fuse", ["1", "0"])
@pytest.mark.parametrize("n_req", [0, 1000, 1001])
def test_label_resident_calls_repeat(n_req, fuse, monkeypatch):
    """HBM-resident plan-label calls back to back.  After the first, a call skips the clear:
    label_kernel writes every result word itself (16 bits per unit, the last word's tail
    zeroed), no statistics atomics run and the dense pass writes the list totals the host
    reads
    (lean calls; KETOGPU_LABEL_FUSE=0: statistics, their reduction and the clear in every
    call).  Every call's answers, the bits past n, the flag words and the per-call
    statistics stay equal — with a host call, another batch and calls with second-stage
    requests in between"""
    monkeypatch.setenv("KETOGPU_UNITS", "label")
    monkeypatch.setenv("KETOGPU_LABEL_FUSE", fuse)
    namespaces, rows, reqs = randgraph.make_family_graph(92)
    snap = Snapshot.from_rows(namespaces, rows, sort=True)
    want = np.asarray(randgraph.oracle_store(namespaces, rows).check_batch(reqs), dtype=bool)
    roots, targets = snap.resolve_many([(ns, o, r, rt.subject_from_dict(x)) for ns, o, r, x in reqs])
    if n_req:
        reps = -(-n_req // len(roots))
        roots, targets, want = (np.tile(x, reps)[:n_req] for x in (roots, targets, want))
    n = len(roots)
    eng = check.Engine(snap)

    def resident_ok(q, w):
        stats = []
        for _ in range(4):
            q.run()
            ab, fb = q.download_words()
            np.testing.assert_array_equal(check.unpack_bits(ab, q.n), w)
            if q.n % 64:
                assert int(ab[-1]) >> (q.n % 64) == 0  # no bit past n
            assert not fb.any()
            st = eng.last_stats()
            assert st["plan"] == 7
            stats.append((st["unit_rows"], st["unit_rev"], st["rest_requests"]))
        # (lean calls collect no statistics: with KETOGPU_LABEL_FUSE=1 every call after the
        # first is one, so compare those)
        assert len(set(stats if fuse == "0" else stats[1:])) == 1, stats
    q = eng.upload(roots, targets)
    resident_ok(q, want)
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)  # a host call in between
    q2 = eng.upload(roots[::-1].copy(), targets[::-1].copy())
    resident_ok(q2, want[::-1])
    resident_ok(q, want)
    # second-stage requests (a quarter of the S heads unlabelled): the clear is never skipped
    monkeypatch.setenv("KETOGPU_LABEL_REST_PERMILLE", "250")
    eng = check.Engine(snap)
    q3 = eng.upload(roots, targets)
    resident_ok(q3, want)
    assert eng.last_stats()["rest_requests"] > 0 and n > 0


@pytest.mark.parametrize("n_req", [1000, 5003, 70000])
def test_label_pipelined_calls(n_req, monkeypatch):
    """ketogpu_queries_run_async: plan-label calls enqueued back to back without a host wait
    (no head unlabelled, no wildcard root: no request can need the second stage), two
    batches interleaved, a host call in between; every batch's bits equal the oracle once
    the engine is waited for.  With unlabelled heads (the test knob) or wildcard roots the
    call runs synchronously and says so"""
    monkeypatch.setenv("KETOGPU_UNITS", "label")
    namespaces, rows, reqs = randgraph.make_family_graph(92)
    snap = Snapshot.from_rows(namespaces, rows, sort=True)
    want = np.asarray(randgraph.oracle_store(namespaces, rows).check_batch(reqs), dtype=bool)
    roots, targets = snap.resolve_many([(ns, o, r, rt.subject_from_dict(x)) for ns, o, r, x in reqs])
    reps = -(-n_req // len(roots))
    roots, targets, want = (np.tile(x, reps)[:n_req] for x in (roots, targets, want))
    eng = check.Engine(snap)
    q = eng.upload(roots, targets)
    q2 = eng.upload(roots[::-1].copy(), targets[::-1].copy())
    q.run()  # (the first call: synchronized, clears)
    queued = [q.run(pipelined=True) for _ in range(3)] + [q2.run(pipelined=True), q.run(pipelined=True)]
    assert all(queued)
    eng.wait()
    np.testing.assert_array_equal(q.download(), want)
    np.testing.assert_array_equal(q2.download(), want[::-1])
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)  # a host call in between
    for _ in range(4):
        assert q2.run(pipelined=True)
    np.testing.assert_array_equal(q2.download(), want[::-1])  # (download waits)
    for _ in range(3):  # each batch's download waits for that batch's call alone
        assert q.run(pipelined=True) and q2.run(pipelined=True)
        np.testing.assert_array_equal(q.download(), want)
        np.testing.assert_array_equal(q2.download(), want[::-1])
    # four batches rotating over the engine's four streams, twice around
    qs = [q, q2, eng.upload(roots, targets), eng.upload(roots[::-1].copy(), targets[::-1].copy())]
    wants = [want, want[::-1], want, want[::-1]]
    for k in range(8):
        assert qs[k % 4].run(pipelined=True)
    for qq, w in zip(qs, wants):
        np.testing.assert_array_equal(qq.download(), w)
    assert eng.last_stats()["plan"] == 7
    # second-stage requests possible: synchronous calls
    monkeypatch.setenv("KETOGPU_LABEL_REST_PERMILLE", "250")
    eng2 = check.Engine(snap)
    q3 = eng2.upload(roots, targets)
    assert not q3.run(pipelined=True)
    np.testing.assert_array_equal(q3.download(), want)
    assert not q3.run(pipelined=True)
    np.testing.assert_array_equal(q3.download(), want)
    assert eng2.last_stats()["rest_requests"] > 0


@pytest.fixture
def global_path(monkeypatch):
    """engines created while active use only the global multi-word path"""
    monkeypatch.setenv("KETOGPU_PATH", "global")


@pytest.mark.parametrize("seed,collide", [(51, False), (52, True), (53, False)])
def test_global_path_matches_oracle(seed, collide, global_path):
    namespaces, rows = randgraph.make_graph(seed, n_rows=800, n_obj=40, n_users=50, poison=True, collide=collide,
                                            empty_ns=True)
    snap = Snapshot.from_rows(namespaces, rows, page_size=4, sort=True)
    eng = check.Engine(snap, max_words_per_round=3)
    orc = randgraph.oracle_store(namespaces, rows, 4)
    reqs = randgraph.make_requests(seed, namespaces, rows, n=1500)
    got = eng.check_many(tuples_of(reqs))
    want = orc.check_batch(reqs)
    assert [g for g in got] == [bool(x) for x in want]
    assert eng.last_stats()["ms_unit"] == 0.0


def test_global_path_small_lists_power_law(global_path):
    # a 1 MiB state budget leaves the minimum frontier lists (65536 entries), so the words
    # per round are bounded by the list capacity (fe_cap / (Ni + 64)) on a graph whose
    # closures are large (Zipf nesting): many rounds, every answer exact
    from keto_amd import synth
    w = synth.social(users=20000, groups=6000, tuples=150000, checks=6000, seed=13)
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    roots, targets = w.resolve(snap)
    want = randgraph.oracle_store_columns(w.namespaces, w.columns).check_batch(
        w.requests(range(len(roots))), nthreads=8)
    eng = check.Engine(snap, state_budget_bytes=1 << 20)
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
    st = eng.last_stats()
    assert st["rounds"] > 1 and st["overflow_retries"] == 0


@pytest.mark.parametrize("path", ["global", "v2"])
@pytest.mark.parametrize("hubs,words", [(64, 0), (256, 3), (1000, 0)])
def test_hub_index(path, hubs, words, monkeypatch):
    # the hub index (searches stop at hubs; the pull reads the hubs' closures) forced on
    # small graphs, on the global path and in the unit2 kernels (whose spills continue on
    # the global path, also with hubs): power-law nesting (hub roots, hubs inside closures,
    # several build rounds) and random tables (wildcards, poisoned pages, dynamic roots)
    from keto_amd import synth
    if path == "global":
        monkeypatch.setenv("KETOGPU_PATH", "global")
    else:
        monkeypatch.setenv("KETOGPU_UNITS", "v2")
    monkeypatch.setenv("KETOGPU_HUBS", str(hubs))
    w = synth.social(users=20000, groups=6000, tuples=150000, checks=8000, seed=17)
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    roots, targets = w.resolve(snap)
    want = randgraph.oracle_store_columns(w.namespaces, w.columns).check_batch(
        w.requests(range(len(roots))), nthreads=8)
    eng = check.Engine(snap, max_words_per_round=words)
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
    st = eng.last_stats()
    assert 0 < st["hubs"] <= hubs
    assert st["plan"] == (0 if path == "global" else 2)
    for seed in (61, 62):
        namespaces, rows = randgraph.make_graph(seed, n_rows=900, n_obj=40, n_users=50, poison=True, empty_ns=True)
        snap = Snapshot.from_rows(namespaces, rows, page_size=4, sort=True)
        orc = randgraph.oracle_store(namespaces, rows, 4)
        reqs = randgraph.make_requests(seed, namespaces, rows, n=1500)
        got = check.Engine(snap, max_words_per_round=words).check_many(tuples_of(reqs))
        assert got == [bool(x) for x in orc.check_batch(reqs)]


def test_hub_index_default_on_power_law(monkeypatch):
    # the default hub selection on a power-law graph: every interior node with >= 8
    # interior successors is a hub; every plan answers as the oracle does
    from keto_amd import synth
    w = synth.social(users=20000, groups=6000, tuples=150000, checks=8000, seed=23)
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    roots, targets = w.resolve(snap)
    want = randgraph.oracle_store_columns(w.namespaces, w.columns).check_batch(
        w.requests(range(len(roots))), nthreads=8)
    for plan in ("bidi", "v2", "lite", "core", "label", "auto"):
        monkeypatch.setenv("KETOGPU_UNITS", plan)
        eng = check.Engine(snap)
        for _ in range(3 if plan == "auto" else 1):
            np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
        st = eng.last_stats()
        if plan in ("label", "auto"):  # the labels answer without searches: no hub index built
            assert st["plan"] == 7 and st["label_on"] == 1 and st["hubs"] == 0
        else:
            assert st["hubs"] > 0


def test_unit_spill_to_global_path(monkeypatch):
    # both sides of the search are n nodes wide: top has n child groups g_i, the target
    # group T is a member of n groups p_i, and only g_7 -> p_7 connects them, so
    # no LDS table holds either side and requests fall through the whole cascade (bidi ->
    # wide bidi -> unit2 -> global path)
    # (g_i expand into u_i and p_i are members of z, so both families are interior nodes);
    # 9000 per side also exceeds the single-request stage's 8192-slot table
    n = 9000
    rows = [(1, "top", "m", None, 1, f"g{i:05d}", "m") for i in range(n)]
    rows += [(1, f"g{i:05d}", "m", f"u{i}", None, None, None) for i in range(n)]
    rows += [(1, f"p{i:05d}", "m", None, 1, "T", "m") for i in range(n)]
    rows += [(1, "z", "m", None, 1, f"p{i:05d}", "m") for i in range(n)]
    rows += [(1, "g00007", "m", None, 1, "p00007", "m")]
    rows += [(1, f"q{i:05d}", "m", None, 1, "T", "m") for i in range(3)]  # T also below q_i only
    snap = Snapshot.from_rows([("n", 1)], rows, sort=True)
    label = check.Engine(snap)  # the default plan: labels answer without a search (nothing spills)
    monkeypatch.setenv("KETOGPU_UNITS", "bidi")
    eng = check.Engine(snap)
    reqs = [rt.InternalRelationTuple("n", "top", "m", rt.SubjectSet("n", "T", "m")),
            rt.InternalRelationTuple("n", "top", "m", rt.SubjectID("u8")),
            rt.InternalRelationTuple("n", "g00009", "m", rt.SubjectSet("n", "T", "m")),  # g_9 -> u9 only
            rt.InternalRelationTuple("n", "q00001", "m", rt.SubjectSet("n", "T", "m")),
            rt.InternalRelationTuple("n", "p00003", "m", rt.SubjectSet("n", "T", "m"))] * 40
    assert label.check_many(reqs) == [True, True, False, True, True] * 40
    assert label.last_stats()["plan"] == 7 and label.last_stats()["spilled_units"] == 0
    got = eng.check_many(reqs)
    assert got == [True, True, False, True, True] * 40
    st = eng.last_stats()
    assert st["spilled_units"] > 0 and st["ms_unit"] > 0
    assert st["spilled_requests"] > 0  # n-wide sides exceed even a single request's table


@pytest.mark.parametrize("plan", ["lite", "bidi"])
def test_lazy_cascade_after_calls_without_spills(monkeypatch, plan):
    """the spill stages are launched after the synchronization when the previous call's
    first stage spilled nothing (device_engine.hip bidi_tail): a batch that spills right
    after batches that did not must still get every answer, from the second pass"""
    n = 9000
    rows = [(1, "top", "m", None, 1, f"g{i:05d}", "m") for i in range(n)]
    rows += [(1, f"g{i:05d}", "m", f"u{i}", None, None, None) for i in range(n)]
    rows += [(1, f"p{i:05d}", "m", None, 1, "T", "m") for i in range(n)]
    rows += [(1, "z", "m", None, 1, f"p{i:05d}", "m") for i in range(n)]
    rows += [(1, "g00007", "m", None, 1, "p00007", "m")]
    snap = Snapshot.from_rows([("n", 1)], rows, sort=True)
    monkeypatch.setenv("KETOGPU_UNITS", plan)
    eng = check.Engine(snap)
    small = [rt.InternalRelationTuple("n", "g00009", "m", rt.SubjectID("u9")),
             rt.InternalRelationTuple("n", "g00009", "m", rt.SubjectID("u8"))] * 50
    wide = [rt.InternalRelationTuple("n", "top", "m", rt.SubjectSet("n", "T", "m")),
            rt.InternalRelationTuple("n", "g00009", "m", rt.SubjectSet("n", "T", "m"))] * 50
    for _ in range(3):
        assert eng.check_many(small) == [True, False] * 50
        assert eng.last_stats()["spilled_units"] == 0
    assert eng.check_many(wide) == [True, False] * 50  # spills: the lazy second pass
    st = eng.last_stats()
    assert st["spilled_units"] > 0
    assert st["unit_launches"] >= 3  # first stage, then the stages and the statistics again
    assert eng.check_many(wide) == [True, False] * 50  # spilled last time: stages up front
    assert eng.check_many(small) == [True, False] * 50


def test_large_forward_closure_small_backward_side():
    # a 14000-group forward closure with a 1-entry backward side: bidi expands the backward
    # side and looks the root's row up, so nothing spills; the forward-only plan spills past
    # even the single-request stage's 12288-node table to the global path
    rows = [(1, "top", "m", None, 1, f"g{i:05d}", "m") for i in range(14000)]
    rows += [(1, f"g{i:05d}", "m", f"u{i}", None, None, None) for i in range(14000)]
    rows += [(1, "small", "m", None, 1, "g00007", "m")]
    snap = Snapshot.from_rows([("n", 1)], rows, sort=True)
    reqs, want = [], []
    for i in range(0, 14000, 233):
        reqs.append(rt.InternalRelationTuple("n", "top", "m", rt.SubjectID(f"u{i}")))
        reqs.append(rt.InternalRelationTuple("n", "small", "m", rt.SubjectID(f"u{i}")))
        want += [True, i == 7]
    assert check.Engine(snap).check_many(reqs) == want
    os.environ["KETOGPU_UNITS"] = "v2"
    try:
        eng = check.Engine(snap)
    finally:
        del os.environ["KETOGPU_UNITS"]
    assert eng.check_many(reqs) == want
    assert eng.last_stats()["spilled_requests"] > 0


def test_check_ids_and_device_queries_match_oracle():
    namespaces, rows = randgraph.make_graph(41, n_rows=3000, n_obj=200, n_rel=3, n_users=300)
    snap = Snapshot.from_rows(namespaces, rows, sort=True)
    orc = randgraph.oracle_store(namespaces, rows)
    reqs = [q for q in randgraph.make_requests(41, namespaces, rows, n=5000, wildcard=False)]
    roots, targets = snap.resolve_many([(ns, o, r, rt.subject_from_dict(s)) for ns, o, r, s in reqs])
    want = orc.check_batch(reqs)
    eng = check.Engine(snap, max_words_per_round=7)  # several rounds
    allowed, flags = eng.check_ids(roots, targets, with_flags=True)
    assert not flags.any()
    np.testing.assert_array_equal(allowed, want)
    q = eng.upload(roots, targets)
    for _ in range(3):  # state must be fully reset between runs
        q.run()
        np.testing.assert_array_equal(q.download(), want)
    st = eng.last_stats()
    assert st["checks"] == len(reqs) and st["bytes_unit"] > 0 and st["ms_total"] > 0
    # (plan label's lean resident calls collect no per-kernel timings or statistics: with
    # timing events on, the same call reports both)
    eng.set_events(True)
    q.run()
    eng.set_events(False)
    np.testing.assert_array_equal(q.download(), want)
    st = eng.last_stats()
    assert st["ms_unit"] > 0 and st["unit_rows"] + st["unit_edges"] + st["unit_rev"] > 0


def test_deep_chain_has_no_depth_cutoff():
    # check has no max-depth (engine.go:93-95): a 3000-long chain of subject sets
    n = 3000
    rows = [(1, f"g{i}", "m", None, 1, f"g{i + 1}", "m") for i in range(n)]
    rows.append((1, f"g{n}", "m", "alice", None, None, None))
    snap = Snapshot.from_rows([("n", 1)], rows, sort=True)
    eng = check.Engine(snap)
    reqs = [rt.InternalRelationTuple("n", f"g{i}", "m", rt.SubjectID("alice")) for i in (0, 1, 1500, n)]
    reqs.append(rt.InternalRelationTuple("n", "g0", "m", rt.SubjectID("bob")))
    reqs.append(rt.InternalRelationTuple("n", "g0", "m", rt.SubjectSet("n", "g0", "m")))  # cycle-free: false
    reqs.append(rt.InternalRelationTuple("n", "g0", "m", rt.SubjectSet("n", f"g{n}", "m")))
    assert eng.check_many(reqs) == [True, True, True, True, False, False, True]


@pytest.mark.parametrize("kind", ["rbac", "folders", "social"])
def test_synthetic_configs_match_oracle(kind, unit_plan):
    """BASELINE configs #2 (RBAC), #3 (folders, depth 10) and #4 (power-law groups) at
    small scale, every request against the oracle"""
    from keto_amd import synth
    w = {"rbac": lambda: synth.rbac(users=20000, groups=2000, docs=4000, tuples=120000, checks=20000, seed=7),
         "folders": lambda: synth.folders(users=8000, groups=300, folders=12000, tuples=150000, checks=20000, seed=7),
         "social": lambda: synth.social(users=20000, groups=6000, tuples=150000, checks=20000, seed=7)}[kind]()
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    orc = randgraph.oracle_store_columns(w.namespaces, w.columns)
    roots, targets = w.resolve(snap)
    eng = check.Engine(snap)
    got = eng.check_ids(roots, targets)
    want = orc.check_batch(w.requests(range(len(roots))), nthreads=8)
    np.testing.assert_array_equal(got, want)
    assert 0.3 < got.mean() < 0.9


def test_loaded_snapshot_answers_identically(tmp_path):
    from keto_amd import synth
    w = synth.rbac(users=20000, groups=2000, docs=4000, tuples=120000, checks=5000, seed=11)
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    snap.save(tmp_path / "rbac.snap")
    back = Snapshot.load(tmp_path / "rbac.snap", w.namespaces)
    roots, targets = w.resolve(snap)
    r2, t2 = w.resolve(back)
    np.testing.assert_array_equal(roots, r2)
    np.testing.assert_array_equal(targets, t2)
    np.testing.assert_array_equal(check.Engine(back).check_ids(roots, targets),
                                  check.Engine(snap).check_ids(roots, targets))


@pytest.mark.parametrize("kind", ["rbac", "folders"])
@pytest.mark.parametrize("labels", [True, False])
def test_auto_plan_trials_then_keeps_one(kind, labels, monkeypatch):
    """KETOGPU_UNITS=auto (default): with plan label's labels built, every call runs plan
    label (no trials); without them (KETOGPU_NO_LABEL) the first two batches of >= 65536
    requests run every candidate first stage and the engine keeps the faster; every call is
    exact"""
    from keto_amd import synth
    monkeypatch.delenv("KETOGPU_UNITS", raising=False)
    if not labels:
        monkeypatch.setenv("KETOGPU_NO_LABEL", "1")
    w = {"rbac": lambda: synth.rbac(users=20000, groups=2000, docs=4000, tuples=120000, checks=70000, seed=9),
         "folders": lambda: synth.folders(users=8000, groups=300, folders=12000, tuples=150000, checks=70000,
                                          seed=9)}[kind]()
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    roots, targets = w.resolve(snap)
    want = randgraph.oracle_store_columns(w.namespaces, w.columns).check_batch(
        w.requests(range(len(roots))), nthreads=8)
    eng = check.Engine(snap)
    np.testing.assert_array_equal(eng.check_ids(roots[:1000], targets[:1000]), want[:1000])
    assert eng.last_stats()["plan"] == (7 if labels else 6)  # below the trial size: label, else core
    plans = set()
    for _ in range(4):
        np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
        plans.add(eng.last_stats()["plan"])
    # label; else the global path (with the hub index), bidi, unit2, lite, core
    assert plans == {7} if labels else plans <= {0, 1, 2, 5, 6}
    kept = eng.last_stats()["plan"]
    np.testing.assert_array_equal(eng.check_ids(roots[:5000], targets[:5000]), want[:5000])
    assert eng.last_stats()["plan"] == kept


@pytest.mark.parametrize("graph,heads", [("random", "0,0"), ("random", "8,8"), ("family", "0,0"), ("family", "8,16"),
                                         ("family-regrow", "0,0"), ("social", "0,0"), ("rbac", "0,0")])
def test_label_device_build_equals_host(graph, heads, monkeypatch):
    """the head arrays an engine builds on the device (label_count / write / patch kernels,
    the host building only the lists of more than 64 entries) equal the host build
    (labels.cpp build_labels, the test hook) word for word; a second engine over the same
    snapshot reuses the snapshot's 2-hop labels (one build) and builds the same arrays"""
    from keto_amd import synth
    if graph == "random":
        namespaces, rows = randgraph.make_graph(33, n_rows=900, n_obj=40, n_users=50, poison=True)  # (no R4 keys)
        snap = Snapshot.from_rows(namespaces, rows, page_size=3, sort=True)
    elif graph.startswith("family"):
        namespaces, rows, _ = randgraph.make_family_graph(92)
        snap = Snapshot.from_rows(namespaces, rows, sort=True)
        if graph == "family-regrow":  # room for one long list at first: the count pass runs again
            monkeypatch.setenv("KETOGPU_TEST_LABEL_BIG_CAP", "1")
    else:
        w = (synth.social(users=20000, groups=6000, tuples=150000, checks=10, seed=7) if graph == "social" else
             synth.rbac(users=20000, groups=2000, docs=4000, tuples=120000, checks=10, seed=7))
        snap = Snapshot.from_columns(w.namespaces, w.columns)
    monkeypatch.setenv("KETOGPU_LABEL_HEADS", heads)
    hs, hp = (int(x) for x in heads.split(","))
    li = snap.label_index(hs, hp)
    engines = [check.Engine(snap), check.Engine(snap)]
    for eng in engines:
        S, hs_dev = eng.label_heads(0)
        P, hp_dev = eng.label_heads(1)
        assert (hs_dev, hp_dev) == (li["s_head_words"], li["p_head_words"])
        np.testing.assert_array_equal(S, li["S"])
        np.testing.assert_array_equal(P, li["P"])
    # one 2-hop label build per snapshot (labels.cpp reach_labels_of): the engines report the
    # same build (its time), which the host hook's own build does not share
    pll = [e.check_ids(np.zeros(1, np.uint32), np.zeros(1, np.uint32)) is not None and e.last_stats()["label_pll_ms"]
           for e in engines]
    assert pll[0] == pll[1] > 0
