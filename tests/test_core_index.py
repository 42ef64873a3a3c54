"""Plan core's record arrays (keto_amd/csrc/core_index.hpp), built on the host as the
engine builds them, against an independent decoding in Python: every node block holds
exactly the node's seed row (fint(v) forward, rev(v) backward, in row order), every record
names the node's expansion row, a closure row is exactly the node's closure (breadth-first
search here over the snapshot's rows), and a node keeps its one-hop row only when its
closure has more nodes than the cap.  CPU only (no device calls)."""
import numpy as np
import pytest

from keto_amd import relationtuple as rt
from keto_amd.snapshot import Snapshot
from tests import randgraph

NONE = 0xFFFFFFFF
TERMINAL, CLOSURE = 0x80000000, 0x40000000


def interior_rows(g, d):
    """one-hop interior rows per interior node: forward fint(v), backward the interior
    predecessors (rev(v) below Ni)"""
    Ni = g["Ni"]
    out = []
    for v in range(Ni):
        if d == 0:
            row = g["fint_col"][g["fint_off"][v]:g["fint_off"][v + 1]]
        else:
            row = g["rev_col"][g["rev_off"][v]:g["rev_off"][v + 1]]
            row = row[row < Ni]
        out.append([int(x) for x in row])
    return out


def closure(rows, v, limit):
    """nodes reachable from v through >= 1 step, without v; None beyond `limit` nodes"""
    seen, order, queue = {v}, [], [v]
    while queue:
        x = queue.pop()
        for y in rows[x]:
            if y not in seen:
                seen.add(y)
                order.append(y)
                if len(order) > limit:
                    return None
                queue.append(y)
    return sorted(order)


def check_index(snap, cap, block=(0, 0)):
    g = snap.graph()
    ci = snap.core_index(cap, block)
    Ni = g["Ni"]
    for d in (0, 1):
        c = ci[d]
        R = c["records"].astype(np.uint64)
        rows = interior_rows(g, d)
        B = c["block_records"]
        assert B in (4, 8, 16, 32) and c["block_base"] % B == 0
        if block[d]:
            assert B == block[d]
        n_clo = n_ent = 0
        expect = {}  # node -> expected record fields (deg/begin checked through the row they name)

        def check_rec(rec):
            u = int(rec[0])
            deg, begin, pad = int(rec[1]), int(rec[2]), int(rec[3])
            if u >= Ni:
                assert (deg, begin, pad) == (0, 0, 0), rec
                return
            if u in expect:
                assert expect[u] == (deg, begin, pad)
                return
            expect[u] = (deg, begin, pad)
            full = closure(rows, u, max(cap[d], 0))
            if pad & CLOSURE:
                got = R[begin:begin + deg]
                assert all(int(x[3]) == TERMINAL and int(x[1]) == 0 and int(x[2]) == 0 for x in got)
                assert [int(x[0]) for x in got] == full, (d, u)
                assert 0 < deg <= cap[d]
            else:
                assert pad == 0
                got = [int(x) for x in R[begin:begin + deg, 0]]
                assert got == rows[u], (d, u)
                # a one-hop row only when the closure is empty or over the cap
                assert full is None or not full or cap[d] == 0, (d, u, full)

        nodes = g["Nx"] if d == 0 else g["N"]
        off, col = (g["fint_off"], g["fint_col"]) if d == 0 else (g["rev_off"], g["rev_col"])
        over = 0
        for v in range(nodes):
            h = R[c["block_base"] + v * B]
            n, first = int(h[0]), int(h[1]) | (int(h[2]) << 32)
            want = [int(x) for x in col[off[v]:off[v + 1]]]
            assert n == len(want)
            if n < B:
                assert first == c["block_base"] + v * B + 1
                tail = R[first + n:c["block_base"] + (v + 1) * B]
                assert all(int(x[0]) == NONE for x in tail)
            else:
                over += 1
                assert first >= c["block_base"] + nodes * B
            got = R[first:first + n]
            assert [int(x[0]) for x in got] == want, (d, v)
            for rec in got:
                check_rec(rec)
        assert over == c["overflow_rows"]
        for v in range(Ni):  # every core and closure row, also of nodes no seed row names
            for rec in R[expect[v][1]:expect[v][1] + expect[v][0]] if v in expect else []:
                if not int(rec[3]) & TERMINAL:
                    check_rec(rec)
        for u, (deg, begin, pad) in expect.items():
            if pad & CLOSURE:
                n_clo += 1
                n_ent += deg
        assert n_clo <= c["closure_nodes"] and n_ent <= c["closure_entries"]
    return ci


@pytest.mark.parametrize("seed,poison,collide", [(71, False, False), (72, True, False), (73, True, True)])
@pytest.mark.parametrize("cap", [(64, 64), (3, 3), (0, 0), (0, 8)])
def test_random_tables(seed, poison, collide, cap):
    namespaces, rows = randgraph.make_graph(seed, n_rows=700, n_obj=40, n_users=40, poison=poison, collide=collide,
                                            empty_ns=True)
    snap = Snapshot.from_rows(namespaces, rows, page_size=5, sort=True)
    check_index(snap, cap)


@pytest.mark.parametrize("block", [(4, 4), (8, 32), (32, 16)])
def test_block_sizes(block):
    namespaces, rows = randgraph.make_graph(74, n_rows=900, n_obj=30, n_users=60)
    snap = Snapshot.from_rows(namespaces, rows, sort=True)
    ci = check_index(snap, (64, 64), block)
    assert ci[0]["block_records"] == block[0] and ci[1]["block_records"] == block[1]


@pytest.mark.parametrize("kind", ["rbac", "folders", "social"])
def test_synthetic_configs(kind):
    """small BASELINE-shaped graphs: RBAC's backward closures (ancestor groups) and the
    folders' forward closures (parent chains) are all within the default cap"""
    from keto_amd import synth
    w = {"rbac": lambda: synth.rbac(users=3000, groups=300, docs=600, tuples=20000, checks=10, seed=5),
         "folders": lambda: synth.folders(users=2000, groups=60, folders=1500, tuples=20000, checks=10, seed=5),
         "social": lambda: synth.social(users=3000, groups=600, tuples=20000, checks=10, seed=5)}[kind]()
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    ci = check_index(snap, (64, 64))
    if kind == "rbac":
        assert ci[1]["closure_nodes"] > 0.9 * snap.graph()["Ni"]
    if kind == "folders":
        assert ci[0]["closure_nodes"] > 0.9 * snap.graph()["Ni"]


def test_cycles():
    """a cycle a -> b -> c -> a and a tail c -> d: the closure of a node on the cycle
    holds the other cycle nodes and d, never the node itself"""
    rows = [(1, "a", "m", None, 1, "b", "m"), (1, "b", "m", None, 1, "c", "m"), (1, "c", "m", None, 1, "a", "m"),
            (1, "c", "m", None, 1, "d", "m"), (1, "d", "m", "u1", None, None, None),
            (1, "a", "m", "u2", None, None, None)]
    snap = Snapshot.from_rows([("n", 1)], rows, sort=True)
    check_index(snap, (64, 64))
    check_index(snap, (2, 2))


# ------------------------------------------------------------------ 2-hop labels
NONE_ = 0xFFFFFFFF


def label_list(A, h, x):
    """(entries, mask) of node x's head in a plan-label head array (labels.hpp), or
    (None, None) for a head marked without label; checks the head's layout"""
    base = x * h
    c, ov = int(A[base]), int(A[base + 1])
    if c == NONE_:
        return None, None
    mask = int(A[base + 2]) | int(A[base + 3]) << 32
    if c <= h - 4:
        lst = A[base + 4: base + 4 + c]
        assert np.all(A[base + 4 + c: base + h] == NONE_)
    else:
        assert ov * 16 + c <= len(A)
        lst = A[ov * 16: ov * 16 + c]
        np.testing.assert_array_equal(A[base + 4: base + h], lst[: h - 4])  # the prefix, also in the head
    assert np.all(np.diff(lst.astype(np.int64)) > 0)
    return lst, mask


def label_answer(li, r, t, ni):
    """allowed(r, t) from plan label's heads (labels.hpp): the masks share a bit, the lists a
    landmark (entries below ni), or a non-interior root r is among S(t)'s raw entries (the
    one-edge test)"""
    if r == NONE_ or t == NONE_:
        return False
    s, sm = label_list(li["S"], li["s_head_words"], t)
    p, pm = label_list(li["P"], li["p_head_words"], r)
    assert np.all(p < ni)  # P lists hold landmarks only
    return bool(sm & pm) or bool(np.isin(p, s[s < ni]).any()) or (r >= ni and r in set(s[s >= ni].tolist()))


def first_stage(li, r, t, ni):
    """the first stage's decision from the two heads alone (device_engine.hip label_unit):
    True / False when the heads settle the request, None when it goes to the dense pass"""
    hs, hp = li["s_head_words"], li["p_head_words"]
    S, P = li["S"], li["P"]
    ns, np_ = int(S[t * hs]), int(P[r * hp])
    sm = int(S[t * hs + 2]) | int(S[t * hs + 3]) << 32
    pm = int(P[r * hp + 2]) | int(P[r * hp + 3]) << 32
    cs, cp = hs - 4, hp - 4
    se = S[t * hs + 4: t * hs + hs].astype(np.int64)  # inline words (0xFFFFFFFF pad)
    pe = P[r * hp + 4: r * hp + hp].astype(np.int64)
    es = int((se < ni).sum())
    ep = min(np_, cp)
    if sm & pm or np.isin(se[:es], pe[:ep]).any() or (r >= ni and (se == r).any()):
        return True
    s_whole = ns <= cs or se[cs - 1] >= ni
    p_whole = np_ <= cp
    s_last = int(se[es - 1]) if es else 0
    p_last = int(pe[ep - 1]) if ep else 0
    lm_done = es == 0 or np_ == 0 or (s_whole and (p_whole or s_last <= p_last)) or (p_whole and p_last <= s_last)
    raw_done = r < ni or ns <= cs or r <= se[cs - 1]
    return False if lm_done and raw_done else None


def check_labels(snap, reqs, want, heads=(0, 0)):
    """every request answered from the heads as the oracle answers it; and wherever the first
    stage's decision from the heads alone settles a request (the prefix rules), it equals
    the oracle too"""
    li = snap.label_index(*heads)
    ni = int(snap.stats()["num_interior"])
    roots, targets = snap.resolve_many([(ns, o, r, rt.subject_from_dict(s)) for ns, o, r, s in reqs])
    settled = 0
    for i in range(len(reqs)):
        r, t = int(roots[i]), int(targets[i])
        assert label_answer(li, r, t, ni) == bool(want[i]), (reqs[i], want[i])
        if r != NONE_ and t != NONE_:
            d = first_stage(li, r, t, ni)
            assert d is None or d == bool(want[i]), (reqs[i], want[i], d)
            settled += d is not None
    li["settled"] = settled
    return li


@pytest.mark.parametrize("seed,poison", [(81, False), (82, True), (83, False), (84, True)])
@pytest.mark.parametrize("heads", [(0, 0), (8, 8), (32, 16)])
def test_labels_answer_like_the_oracle(seed, poison, heads):
    """every request (random tables with cycles, collisions of page sizes, poisoned pages) is
    answered by one intersection exactly as the reference's recursion (oracle), with the
    head sizes chosen from the lists and forced small (most lists in the overflow region)"""
    namespaces, rows = randgraph.make_graph(seed, n_rows=900, n_obj=40, n_users=50, poison=poison)
    snap = Snapshot.from_rows(namespaces, rows, page_size=4, sort=True)
    reqs = randgraph.make_requests(seed, namespaces, rows, n=1500, wildcard=False)
    want = randgraph.oracle_store(namespaces, rows, 4).check_batch(reqs)
    assert any(want) and not all(want)
    li = check_labels(snap, reqs, want, heads)
    if heads != (0, 0):
        assert (li["s_head_words"], li["p_head_words"]) == heads
    else:
        assert li["s_head_words"] in (8, 16, 32, 64) and li["p_head_words"] in (8, 16, 32, 64)
    if heads == (8, 8):
        assert li["s_overflow"] > 0


@pytest.mark.parametrize("seed", [81, 82])
@pytest.mark.parametrize("heads", [(8, 8), (16, 8), (8, 16), (64, 64)])
def test_label_first_stage_decisions(seed, heads):
    """the first stage settles a request from its two heads alone when no landmark can be
    missing from the inline prefixes (both landmark lists whole, or one whole with its largest
    entry <= the other's last inline entry) and the one-edge test is settled (r interior, S
    whole, or r <= S's last inline entry): with small heads most lists overflow and the prefix
    rules decide; every settled request equals the oracle, and P lists hold no raw entry"""
    namespaces, rows = randgraph.make_graph(seed, n_rows=900, n_obj=40, n_users=50, poison=True)
    snap = Snapshot.from_rows(namespaces, rows, page_size=4, sort=True)
    reqs = randgraph.make_requests(seed, namespaces, rows, n=1500, wildcard=False)
    want = randgraph.oracle_store(namespaces, rows, 4).check_batch(reqs)
    li = check_labels(snap, reqs, want, heads)
    assert li["settled"] > 0
    if heads == (64, 64):
        assert li["s_overflow"] == 0 or li["settled"] > 0.9 * len(reqs)


@pytest.mark.parametrize("kind", ["rbac", "folders", "social"])
def test_labels_on_synthetic_configs(kind):
    """configs #2, #3 and #4 (the power-law shape that closure labels could not reach):
    every request is labelled and exact"""
    from keto_amd import synth
    w = {"rbac": lambda: synth.rbac(users=4000, groups=400, docs=800, tuples=30000, checks=3000, seed=6),
         "folders": lambda: synth.folders(users=3000, groups=80, folders=2000, tuples=30000, checks=3000, seed=6),
         "social": lambda: synth.social(users=4000, groups=3000, tuples=40000, checks=3000, seed=6)}[kind]()
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    li = snap.label_index()
    roots, targets = w.resolve(snap)
    ni = int(snap.stats()["num_interior"])
    want = randgraph.oracle_store_columns(w.namespaces, w.columns).check_batch(w.requests(range(len(roots))),
                                                                                 nthreads=4)
    got = [label_answer(li, int(roots[i]), int(targets[i]), ni) for i in range(len(roots))]
    assert got == [bool(x) for x in want]
    assert any(want) and not all(want)
    dec = [first_stage(li, int(roots[i]), int(targets[i]), ni) for i in range(len(roots))
           if roots[i] != NONE_ and targets[i] != NONE_]
    assert all(d is None or d == bool(x) for d, x in zip(dec, [w_ for i, w_ in enumerate(want)
                                                              if roots[i] != NONE_ and targets[i] != NONE_]))
    # the head size rule (labels.cpp pick_head): 64 words where they hold >= 10% more of the
    # lists inline than 32; a smaller head only where it holds as many as 32 (within 0.1%)
    for A, h, n in ((li["S"], li["s_head_words"], li["s_nodes"]), (li["P"], li["p_head_words"], li["p_nodes"])):
        c = A[: n * h].reshape(-1, h)[:, 0].astype(np.int64)
        c = c[c > 0]
        if len(c) == 0:
            continue
        fit32, fit64 = (c <= 28).mean(), (c <= 60).mean()
        assert h in (8, 16, 32, 64)
        assert (h == 64) == (fit64 - fit32 >= 0.1)
        if h < 32:
            assert (c <= h - 4).mean() >= 0.999 * fit32


def test_long_lists():
    """nodes whose lists pass every head size (the family graph's wide closures): kept
    whole in the overflow region and answered exactly"""
    namespaces, rows, reqs = randgraph.make_family_graph(91)
    snap = Snapshot.from_rows(namespaces, rows, sort=True)
    want = randgraph.oracle_store(namespaces, rows).check_batch(reqs)
    assert any(want) and not all(want)
    li = check_labels(snap, reqs, want, (8, 8))
    assert li["s_overflow"] > 0 and li["label_entries"] > 0


def test_labels_on_a_written_writable_snapshot():
    """a writable snapshot's rows end in free slots (placeholder nodes): the labels are
    built from the real entries only, and answer every request exactly after writes"""
    from tests.test_writes import _graph, _writes, _expected, _sqlite_key
    namespaces, rows = _graph(341, n_rows=700, n_obj=25, n_users=30)
    w = Snapshot.from_rows(namespaces, rows, sort=True, writable=True)
    cur = sorted(rows, key=_sqlite_key)
    for step in range(3):
        ins, dele = _writes(600 + step, namespaces, cur)
        assert w.write(ins, dele)["applied"]
        cur = _expected(cur, ins, dele)
        reqs = randgraph.make_requests(700 + step, namespaces, cur, n=800, wildcard=False)
        want = randgraph.oracle_store(namespaces, cur).check_batch(reqs)
        check_labels(w, reqs, want)
