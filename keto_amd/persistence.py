"""SQL persistence side: the keto_relation_tuples table (SQLite) and the snapshot
loader that streams it, ordered, into libketogpu's builder.

Mirrors internal/persistence/sql:
  schema               migrations/templates/20210623162417_relationtuple.up.sql:3-48
  InsertRelationTuple  relationtuples.go:82-149 (names -> namespace ids)
  ORDER BY             relationtuples.go:215
  nid filter           persister.go:117-119
The loader replaces per-node GetRelationTuples calls: ONE ordered SELECT per network,
read in batches (the backend's own ordering and collation are captured, R9).
"""
import sqlite3
import uuid

import numpy as np

from . import relationtuple as rt

ORDER_BY = ("nid, namespace_id, object, relation, subject_id, subject_set_namespace_id, subject_set_object, "
            "subject_set_relation, commit_time")
# Postgres executes the same ORDER BY with NULLs last (ASC); SQLite >= 3.30 states that
# with NULLS LAST, so a SQLite table can serve rows in a Postgres ("C" collation) order.
ORDER_BY_NULLS_LAST = ("nid, namespace_id, object, relation, subject_id NULLS LAST, "
                       "subject_set_namespace_id NULLS LAST, subject_set_object NULLS LAST, "
                       "subject_set_relation NULLS LAST, commit_time")


def order_by(order="sqlite"):
    """the ORDER BY clause of relationtuples.go:215 as backend `order` executes it"""
    return ORDER_BY_NULLS_LAST if order == "postgres" else ORDER_BY

SCHEMA = """
CREATE TABLE IF NOT EXISTS keto_relation_tuples
(
    shard_id                 UUID        NOT NULL,
    nid                      UUID        NOT NULL,
    namespace_id             INTEGER     NOT NULL,
    object                   VARCHAR(64) NOT NULL,
    relation                 VARCHAR(64) NOT NULL,
    subject_id               VARCHAR(64) NULL,
    subject_set_namespace_id INTEGER NULL,
    subject_set_object       VARCHAR(64) NULL,
    subject_set_relation     VARCHAR(64) NULL,
    commit_time              TIMESTAMP   NOT NULL,
    PRIMARY KEY (shard_id, nid),
    CONSTRAINT chk_keto_rt_subject_type CHECK
        ((subject_id IS NULL AND
          subject_set_namespace_id IS NOT NULL AND subject_set_object IS NOT NULL AND subject_set_relation IS NOT NULL)
            OR
         (subject_id IS NOT NULL AND
          subject_set_namespace_id IS NULL AND subject_set_object IS NULL AND subject_set_relation IS NULL))
);
CREATE INDEX IF NOT EXISTS keto_relation_tuples_full_idx ON keto_relation_tuples (nid, namespace_id, object,
    relation, subject_id, subject_set_namespace_id, subject_set_object, subject_set_relation, commit_time);
"""


class UnknownNamespace(LookupError):
    """herodot.ErrNotFound for an unknown namespace name/id"""


class TupleStore:
    """keto_relation_tuples of one network (nid) plus the namespace configuration."""

    def __init__(self, namespaces, conn=None, nid=None, page_size=100, order="sqlite"):
        self.conn = conn or sqlite3.connect(":memory:")
        self.conn.executescript(SCHEMA)
        self.namespaces = [(n, i) for n, i in namespaces]  # config order
        self.nid = nid or str(uuid.uuid4())
        self.page_size = page_size
        self.order = order  # the backend whose row order reads emulate (order_by)
        self._ct = 0

    # namespace_memory.go:29-47 (first match)
    def ns_id(self, name):
        for n, i in self.namespaces:
            if n == name:
                return i
        raise UnknownNamespace(name)

    def insert(self, t: rt.InternalRelationTuple, commit_time=None):
        if t.subject is None:
            raise rt.NilSubject()
        if commit_time is None:
            commit_time = self._ct
        self._ct += 1
        nsid = self.ns_id(t.namespace)
        if isinstance(t.subject, rt.SubjectID):
            vals = (t.subject.id, None, None, None)
        else:
            vals = (None, self.ns_id(t.subject.namespace), t.subject.object, t.subject.relation)
        self.conn.execute(
            "INSERT INTO keto_relation_tuples (shard_id, nid, namespace_id, object, relation, subject_id, "
            "subject_set_namespace_id, subject_set_object, subject_set_relation, commit_time) "
            "VALUES (?,?,?,?,?,?,?,?,?,?)",
            (str(uuid.uuid4()), self.nid, nsid, t.object, t.relation) + vals + (commit_time,))

    def insert_raw(self, namespace_id, obj, rel, subject_id=None, ss_ns=None, ss_obj=None, ss_rel=None,
                   commit_time=None):
        """a row with arbitrary namespace ids (e.g. ids later removed from the config)"""
        if commit_time is None:
            commit_time = self._ct
        self._ct += 1
        self.conn.execute(
            "INSERT INTO keto_relation_tuples (shard_id, nid, namespace_id, object, relation, subject_id, "
            "subject_set_namespace_id, subject_set_object, subject_set_relation, commit_time) "
            "VALUES (?,?,?,?,?,?,?,?,?,?)",
            (str(uuid.uuid4()), self.nid, namespace_id, obj, rel, subject_id, ss_ns, ss_obj, ss_rel, commit_time))

    def iter_ordered_batches(self, batch_rows=1 << 16):
        """the loader's single ordered read, as columnar batches (ketogpu_row_batch)"""
        cur = self.conn.execute(
            "SELECT namespace_id, object, relation, subject_id, subject_set_namespace_id, subject_set_object, "
            f"subject_set_relation FROM keto_relation_tuples WHERE nid = ? ORDER BY {order_by(self.order)}",
            (self.nid,))
        while True:
            rows = cur.fetchmany(batch_rows)
            if not rows:
                return
            yield columnar(rows)


def _strcol(vals):
    enc = [(v or "").encode("utf-8") for v in vals]
    off = np.zeros(len(enc) + 1, dtype=np.uint64)
    if enc:
        off[1:] = np.cumsum([len(e) for e in enc], dtype=np.uint64)
    data = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8).copy()
    return data, off


def columnar(rows):
    """[(namespace_id, object, relation, subject_id|None, ss_ns|None, ss_obj, ss_rel)] -> column dict"""
    n = len(rows)
    cols = {"namespace_id": np.array([r[0] for r in rows], dtype=np.int32)}
    cols["object_data"], cols["object_off"] = _strcol([r[1] for r in rows])
    cols["relation_data"], cols["relation_off"] = _strcol([r[2] for r in rows])
    kind = np.array([0 if r[3] is not None else 1 for r in rows], dtype=np.uint8)
    cols["subject_kind"] = kind
    cols["subject_id_data"], cols["subject_id_off"] = _strcol([r[3] if r[3] is not None else "" for r in rows])
    cols["ss_namespace_id"] = np.array([r[4] if r[4] is not None else 0 for r in rows], dtype=np.int32)
    cols["ss_object_data"], cols["ss_object_off"] = _strcol([r[5] for r in rows])
    cols["ss_relation_data"], cols["ss_relation_off"] = _strcol([r[6] for r in rows])
    cols["commit_time"] = np.arange(n, dtype=np.int64)
    return cols


def rows_from_tuples(namespaces, tuples):
    """fixture tuples (dicts or InternalRelationTuple) -> raw rows, names resolved to ids"""
    def nsid(name):
        for n, i in namespaces:
            if n == name:
                return i
        raise UnknownNamespace(name)

    out = []
    for t in tuples:
        if isinstance(t, dict):
            t = rt.InternalRelationTuple.from_dict(t)
        if isinstance(t.subject, rt.SubjectID):
            out.append((nsid(t.namespace), t.object, t.relation, t.subject.id, None, None, None))
        else:
            s = t.subject
            out.append((nsid(t.namespace), t.object, t.relation, None, nsid(s.namespace), s.object, s.relation))
    return out


def request_columns(requests):
    """check requests [(namespace, object, relation, subject)] -> ketogpu_request_batch
    columns (subject: SubjectID, SubjectSet, None for nil, or their dict forms)"""
    subs = [rt.subject_from_dict(q[3]) if isinstance(q[3], dict) else q[3] for q in requests]
    cols = {"n": len(requests)}
    cols["ns_data"], cols["ns_off"] = _strcol([q[0] for q in requests])
    cols["obj_data"], cols["obj_off"] = _strcol([q[1] for q in requests])
    cols["rel_data"], cols["rel_off"] = _strcol([q[2] for q in requests])
    cols["subject_kind"] = np.array([255 if s is None else 0 if isinstance(s, rt.SubjectID) else 1 for s in subs],
                                    dtype=np.uint8)
    cols["sid_data"], cols["sid_off"] = _strcol([s.id if isinstance(s, rt.SubjectID) else "" for s in subs])
    ss = [s if isinstance(s, rt.SubjectSet) else rt.SubjectSet() for s in subs]
    cols["ss_ns_data"], cols["ss_ns_off"] = _strcol([x.namespace for x in ss])
    cols["ss_obj_data"], cols["ss_obj_off"] = _strcol([x.object for x in ss])
    cols["ss_rel_data"], cols["ss_rel_off"] = _strcol([x.relation for x in ss])
    return cols
