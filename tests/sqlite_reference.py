"""Second, independent restatement of the reference engines over a REAL SQLite
database (test-only).  It issues the reference's own SQL (filters, ORDER BY,
LIMIT/OFFSET plus pop's COUNT) so ordering, NULL placement, collation and
pagination come from sqlite3 itself rather than from our C oracle.  Used to
cross-check oracle/keto_oracle.c on random graphs.

Restates: internal/persistence/sql/relationtuples.go:43-80,203-258,
internal/persistence/sql/persister.go:129-157, internal/check/engine.go:33-95,
internal/expand/engine.go:30-98, internal/x/graph/graph_utils.go:13-35.
"""
import sqlite3

from keto_amd import persistence

ORDER = persistence.ORDER_BY


class NotFound(Exception):
    pass


class SqliteReference:
    def __init__(self, db: persistence.TupleStore):
        self.db = db
        self.conn = db.conn
        self.page_size = db.page_size
        self.order = getattr(db, "order", "sqlite")

    # internal/driver/config/namespace_memory.go:29-47
    def ns_by_name(self, name):
        for n, i in self.db.namespaces:
            if n == name:
                return i
        raise NotFound(name)

    def ns_by_id(self, nid):
        for n, i in self.db.namespaces:
            if i == nid:
                return n
        raise NotFound(nid)

    # GetRelationTuples, relationtuples.go:203-258
    def get_relation_tuples(self, ns, obj, rel, page):
        where, args = ["nid = ?"], [self.db.nid]
        if rel:
            where.append("relation = ?")
            args.append(rel)
        if obj:
            where.append("object = ?")
            args.append(obj)
        if ns:
            where.append("namespace_id = ?")
            args.append(self.ns_by_name(ns))
        w = " AND ".join(where)
        total = self.conn.execute(f"SELECT COUNT(*) FROM keto_relation_tuples WHERE {w}", args).fetchone()[0]
        ps = self.page_size
        rows = self.conn.execute(
            f"SELECT namespace_id, object, relation, subject_id, subject_set_namespace_id, subject_set_object, "
            f"subject_set_relation FROM keto_relation_tuples WHERE {w} ORDER BY {persistence.order_by(self.order)} "
            f"LIMIT ? OFFSET ?",
            args + [ps, (page - 1) * ps]).fetchall()
        total_pages = (total + ps - 1) // ps
        has_next = page < total_pages
        out = []
        for nsid, o, r, sid, ssns, ssobj, ssrel in rows:  # toInternal
            self.ns_by_id(nsid)
            if sid is not None:
                out.append(("id", sid))
            else:
                out.append(("set", self.ns_by_id(ssns), ssobj, ssrel))
        return out, has_next

    @staticmethod
    def key(s):
        return s[1] if s[0] == "id" else f"{s[1]}:{s[2]}#{s[3]}"

    def check(self, ns, obj, rel, subject):
        return self._one_further(None, subject, ns, obj, rel)

    def _one_further(self, visited, req, ns, obj, rel):
        page = 1
        while True:
            try:
                rels, has_next = self.get_relation_tuples(ns, obj, rel, page)
            except NotFound:
                return False
            allowed = self._allowed(visited, req, rels)
            if allowed or not has_next:
                return allowed
            page += 1

    def _allowed(self, visited, req, rels):
        for sr in rels:
            k = self.key(sr)
            if visited is None:
                child = {k}
            else:
                if k in visited:
                    continue
                visited.add(k)
                child = visited
            if req == sr:
                return True
            if sr[0] != "set":
                continue
            if self._one_further(child, req, sr[1], sr[2], sr[3]):
                return True
        return False

    def expand(self, subject, depth):
        self._visited = None
        return self._build(subject, depth)

    def _build(self, subject, depth):
        if depth <= 0:
            return None
        if subject[0] != "set":
            return {"type": "leaf", "subject_id": subject[1]}
        k = self.key(subject)
        if self._visited is None:
            self._visited = {k}
        elif k in self._visited:
            return None
        else:
            self._visited.add(k)
        node = {"type": "union", "children": []}
        page = 1
        while True:
            rels, has_next = self.get_relation_tuples(subject[1], subject[2], subject[3], page)
            if not rels:
                return None
            if depth <= 1:
                node = {"type": "leaf"}
                break
            for r in rels:
                c = self._build(r, depth - 1)
                if c is None:
                    c = leaf_of(r)
                node["children"].append(c)
            if not has_next:
                break
            page += 1
        node.update(subject_fields(subject))
        if not node.get("children"):
            node.pop("children", None)
        return node


def subject_fields(s):
    if s[0] == "id":
        return {"subject_id": s[1]}
    return {"subject_set": {"namespace": s[1], "object": s[2], "relation": s[3]}}


def leaf_of(s):
    d = {"type": "leaf"}
    d.update(subject_fields(s))
    return d


def as_tuple_subject(d):
    if d.get("subject_id") is not None:
        return ("id", d["subject_id"])
    s = d["subject_set"]
    return ("set", s["namespace"], s["object"], s["relation"])
