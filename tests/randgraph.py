"""Seeded random relation-tuple tables and requests for parity tests.

Rows are raw keto_relation_tuples rows (namespace ids, not names) so tests can
include ids that are not configured (page poisoning, R7).  `collide=True` uses
names containing ':' and '#' so distinct subjects share Subject.String() keys (R4).
"""
import random


def make_graph(seed, n_rows=200, n_obj=12, n_rel=3, n_users=10, wildcard=True, poison=False, collide=False,
               empty_ns=False, n_ns=3):
    rng = random.Random(seed)
    ns_names = [f"n{i}" for i in range(n_ns)]
    if collide:
        ns_names = ["a", "a:b", "c"][:max(n_ns, 2)]
    if empty_ns:
        ns_names[-1] = ""
    namespaces = [(name, i + 1) for i, name in enumerate(ns_names)]
    ids = [i for _, i in namespaces]
    objs = [f"o{i}" for i in range(n_obj)]
    rels = [f"r{i}" for i in range(n_rel)]
    users = [f"u{i}" for i in range(n_users)]
    if collide:
        objs = objs[: n_obj - 3] + ["b:c", "c", "b"]
        rels = rels[: n_rel - 1] + ["c#d"] if n_rel > 1 else rels
        users = users[: n_users - 3] + ["a:b#c", "a:b:c#r0", "a:b#r0"]
    rows = []
    for _ in range(n_rows):
        ns = rng.choice(ids)
        if poison and rng.random() < 0.03:
            ns = 99  # namespace id that is not configured
        o, r = rng.choice(objs), rng.choice(rels)
        if rng.random() < 0.45:
            rows.append((ns, o, r, rng.choice(users), None, None, None))
        else:
            so = rng.choice(objs)
            sr = rng.choice(rels)
            if wildcard and rng.random() < 0.06:
                so = ""
            if wildcard and rng.random() < 0.06:
                sr = ""
            sns = rng.choice(ids)
            if poison and rng.random() < 0.03:
                sns = 98
            rows.append((ns, o, r, None, sns, so, sr))
    return namespaces, rows


def make_family_graph(seed, families=12, chain=35, docs=3, users=300):
    """groups in chains (family f: g{f}_0 member of g{f}_1 ... of g{f}_{chain-1}), a few
    documents per family viewable by members of a chain group, users members of the chain
    bottoms of 1..4 families: a user's backward label (plan label mode B) holds the chain's
    groups of each of its families (35, 70, 105, 140 nodes), so labels of 33..63, 64..127
    (searched in the S block in place) and none (> 127) all occur.  -> (namespaces, rows, requests)"""
    rng = random.Random(seed)
    rows = []
    for f in range(families):
        for k in range(chain - 1):
            rows.append((1, f"g{f}_{k + 1}", "member", None, 1, f"g{f}_{k}", "member"))
        for d in range(docs):
            rows.append((1, f"d{f}_{d}", "view", None, 1, f"g{f}_{rng.randrange(chain)}", "member"))
    for u in range(users):
        for f in rng.sample(range(families), 1 + u % 4):
            rows.append((1, f"g{f}_0", "member", f"u{u}", None, None, None))
    reqs = []
    for _ in range(4 * users):
        f = rng.randrange(families)
        o, r = (f"d{f}_{rng.randrange(docs)}", "view") if rng.random() < 0.4 else (f"g{f}_{rng.randrange(chain)}",
                                                                                  "member")
        reqs.append(("n", o, r, {"subject_id": f"u{rng.randrange(users)}"}))
    return [("n", 1)], rows, reqs


def make_requests(seed, namespaces, rows, n=300, wildcard=True):
    rng = random.Random(seed + 7)
    names = [n for n, _ in namespaces] + ["unknown"]
    objs = sorted({r[1] for r in rows}) or ["o0"]
    rels = sorted({r[2] for r in rows}) or ["r0"]
    sids = sorted({r[3] for r in rows if r[3] is not None}) or ["u0"]
    sets = sorted({(r[4], r[5], r[6]) for r in rows if r[3] is None})
    id2name = {i: n for n, i in namespaces}
    reqs = []
    for _ in range(n):
        ns, o, r = rng.choice(names), rng.choice(objs), rng.choice(rels)
        if wildcard and rng.random() < 0.05:
            o = ""
        if wildcard and rng.random() < 0.05:
            r = ""
        if wildcard and rng.random() < 0.03:
            ns = ""
        if sets and rng.random() < 0.3:
            sns, so, sr = rng.choice(sets)
            subj = {"subject_set": {"namespace": id2name.get(sns, "unknown"), "object": so, "relation": sr}}
        elif rng.random() < 0.05:
            subj = {"subject_id": "nobody"}
        else:
            subj = {"subject_id": rng.choice(sids)}
        reqs.append((ns, o, r, subj))
    return reqs


def oracle_store_columns(namespaces, cols, page_size=100, presorted=True):
    from oracle import oracle as O
    st = O.Store(namespaces, page_size)
    st.add_columnar(cols)
    return st.finalize(presorted=presorted)


def oracle_store(namespaces, rows, page_size=100, order="sqlite"):
    from oracle import oracle as O
    st = O.Store(namespaces, page_size, order=order)
    for (ns, o, r, sid, sns, so, sr) in rows:
        if sid is not None:
            st.add_row(ns, o, r, subject_id=sid)
        else:
            st.add_row(ns, o, r, ss_ns_id=sns, ss_obj=so, ss_rel=sr)
    return st.finalize()


def backend_sorted(rows, order="sqlite"):
    """rows as the backend returns them for the reference's ORDER BY (relationtuples.go:215),
    bytewise strings; NULLs first (sqlite) or last (postgres).  Stable: equal rows keep
    their insertion (commit_time) order."""
    def key(r):
        ns, o, rel, sid, sns, so, sr = r
        null_sid = sid is None
        first = null_sid if order == "postgres" else not null_sid  # False sorts first
        return (ns, o.encode(), rel.encode(), first, (sid or "").encode(), sns or 0, (so or "").encode(),
                (sr or "").encode())
    return sorted(rows, key=key)
