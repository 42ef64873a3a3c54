"""Snapshot of keto_relation_tuples for one network, built by libketogpu.

The persistence-side loader of DESIGN.md: rows arrive in the backend's ORDER BY
order (internal/persistence/sql/relationtuples.go:215) and become the ordered host
rows (expand) plus the device graph (check).
"""
import ctypes as C

import numpy as np

from . import _lib as L
from . import persistence
from .relationtuple import SubjectID, SubjectSet


def _ptr(a):
    return None if a is None else a.ctypes.data


def subject_struct(subject):
    if subject is None:
        return L.Subject(L.SUBJECT_NIL, None, None, None, None)
    if isinstance(subject, SubjectID):
        return L.Subject(L.SUBJECT_ID, L.b(subject.id), None, None, None)
    return L.Subject(L.SUBJECT_SET, None, L.b(subject.namespace), L.b(subject.object), L.b(subject.relation))


class Snapshot:
    """`order` names the backend whose ORDER BY the rows follow (include/ketogpu.h
    KETOGPU_ORDER_*): "sqlite" (default), "mysql-bin", "cockroach" (NULLs first) or
    "postgres" (NULLs last); it decides where sorting and apply() place rows."""

    def __init__(self, namespaces, page_size=100, sort=False, order="sqlite", writable=False):
        self.L = L.lib()
        self.namespaces = [(n, int(i)) for n, i in namespaces]
        arr = (L.Namespace * max(len(self.namespaces), 1))(*[L.Namespace(i, L.b(n)) for n, i in self.namespaces])
        opts = L.BuildOpts(page_size, (L.BUILD_SORT if sort else 0) | L.ORDERS[order] |
                           (L.BUILD_WRITABLE if writable else 0))
        h = C.c_void_p()
        L.check(self.L.ketogpu_builder_new(arr, len(self.namespaces), C.byref(opts), C.byref(h)))
        self._builder = h
        self.h = None

    def append(self, cols):
        keep = cols  # arrays must stay alive during the call
        rb = L.RowBatch(len(cols["namespace_id"]), _ptr(cols["namespace_id"]), _ptr(cols["object_data"]),
                        _ptr(cols["object_off"]), _ptr(cols["relation_data"]), _ptr(cols["relation_off"]),
                        _ptr(cols["subject_kind"]), _ptr(cols["subject_id_data"]), _ptr(cols["subject_id_off"]),
                        _ptr(cols["ss_namespace_id"]), _ptr(cols["ss_object_data"]), _ptr(cols["ss_object_off"]),
                        _ptr(cols["ss_relation_data"]), _ptr(cols["ss_relation_off"]))
        L.check(self.L.ketogpu_builder_append(self._builder, C.byref(rb)))
        del keep
        return self

    def finish(self):
        h = C.c_void_p()
        b, self._builder = self._builder, None
        L.check(self.L.ketogpu_builder_finish(b, C.byref(h)))
        self.h = h
        return self

    def __del__(self):
        lib = getattr(self, "L", None)
        if lib is None:
            return
        if getattr(self, "_builder", None):
            lib.ketogpu_builder_free(self._builder)
        if getattr(self, "h", None):
            lib.ketogpu_snapshot_free(self.h)
            self.h = None

    # ---- constructors
    @classmethod
    def from_store(cls, store: persistence.TupleStore, batch_rows=1 << 16):
        s = cls(store.namespaces, store.page_size, order=getattr(store, "order", "sqlite"))
        for cols in store.iter_ordered_batches(batch_rows):
            s.append(cols)
        return s.finish()

    @classmethod
    def from_rows(cls, namespaces, rows, page_size=100, sort=True, order="sqlite", writable=False):
        s = cls(namespaces, page_size, sort=sort, order=order, writable=writable)
        if rows:
            s.append(persistence.columnar(rows))
        return s.finish()

    @classmethod
    def from_tuples(cls, namespaces, tuples, page_size=100, writable=False):
        return cls.from_rows(namespaces, persistence.rows_from_tuples(namespaces, tuples), page_size, sort=True,
                             writable=writable)

    @classmethod
    def from_columns(cls, namespaces, cols, page_size=100, sort=False, order="sqlite", writable=False):
        s = cls(namespaces, page_size, sort=sort, order=order, writable=writable)
        s.append(cols)
        return s.finish()

    # ---- freshness (ketogpu_snapshot_apply / ketogpu_snapshot_write)
    @staticmethod
    def _batch(rows):
        if not rows:
            return None, None
        cols = persistence.columnar(list(rows))
        rb = L.RowBatch(len(rows), _ptr(cols["namespace_id"]), _ptr(cols["object_data"]), _ptr(cols["object_off"]),
                        _ptr(cols["relation_data"]), _ptr(cols["relation_off"]), _ptr(cols["subject_kind"]),
                        _ptr(cols["subject_id_data"]), _ptr(cols["subject_id_off"]),
                        _ptr(cols["ss_namespace_id"]), _ptr(cols["ss_object_data"]), _ptr(cols["ss_object_off"]),
                        _ptr(cols["ss_relation_data"]), _ptr(cols["ss_relation_off"]))
        return rb, cols

    def write(self, insert_rows=(), delete_rows=()):
        """in-place write on a writable snapshot (ketogpu_snapshot_write): the same batch
        semantics as apply(); returns the result dict — "applied" False (with a "reason")
        leaves the snapshot unchanged and the caller rebuilds with apply()"""
        ins, keep_i = self._batch(insert_rows)
        dele, keep_d = self._batch(delete_rows)
        res = L.WriteResult()
        L.check(self.L.ketogpu_snapshot_write(self.h, C.byref(ins) if ins else None, C.byref(dele) if dele else None,
                                              C.byref(res)))
        del keep_i, keep_d
        return res.as_dict()

    def version(self):
        """writes applied in place so far"""
        return int(self.L.ketogpu_snapshot_version(self.h))

    def apply(self, insert_rows=(), delete_rows=()):
        """the next version: raw rows (namespace_id, object, relation, subject_id|None, ss_ns,
        ss_obj, ss_rel) inserted, then every row matching a delete removed"""
        ins, keep_i = self._batch(insert_rows)
        dele, keep_d = self._batch(delete_rows)
        h = C.c_void_p()
        L.check(self.L.ketogpu_snapshot_apply(self.h, C.byref(ins) if ins else None, C.byref(dele) if dele else None,
                                              C.byref(h)))
        del keep_i, keep_d
        s = Snapshot.__new__(Snapshot)
        s.L, s.namespaces, s._builder, s.h = self.L, list(self.namespaces), None, h
        return s

    def set_namespaces(self, namespaces):
        """the next version under a new namespace configuration (ketogpu_snapshot_set_namespaces;
        Keto's KeyNamespaces reload, internal/driver/config/provider.go:87-110)"""
        ns = [(n, int(i)) for n, i in namespaces]
        arr = (L.Namespace * max(len(ns), 1))(*[L.Namespace(i, L.b(n)) for n, i in ns])
        h = C.c_void_p()
        L.check(self.L.ketogpu_snapshot_set_namespaces(self.h, arr, len(ns), C.byref(h)))
        s = Snapshot.__new__(Snapshot)
        s.L, s.namespaces, s._builder, s.h = self.L, ns, None, h
        return s

    # ---- persistence (ketogpu_snapshot_save / _load)
    def save(self, path):
        L.check(self.L.ketogpu_snapshot_save(self.h, str(path).encode()))

    @classmethod
    def load(cls, path, namespaces=None):
        """a snapshot written by save(); `namespaces` only labels the Python object"""
        s = cls.__new__(cls)
        s.L = L.lib()
        s.namespaces = list(namespaces or [])
        s._builder = None
        h = C.c_void_p()
        L.check(s.L.ketogpu_snapshot_load(str(path).encode(), C.byref(h)))
        s.h = h
        return s

    # ---- queries
    def stats(self):
        st = L.SnapshotStats()
        L.check(self.L.ketogpu_snapshot_stats_get(self.h, C.byref(st)))
        return st.as_dict()

    def graph(self):
        """numpy copies of the device graph (ketogpu_snapshot_graph)"""
        v = L.GraphView()
        L.check(self.L.ketogpu_snapshot_graph(self.h, C.byref(v)))
        nx, n = v.num_expandable, v.num_nodes
        fo = np.ctypeslib.as_array(v.fint_off, (nx + 1,)).copy()
        ro = np.ctypeslib.as_array(v.rev_off, (n + 1,)).copy()
        def col(ptr, n):  # an empty column may have no storage
            return np.ctypeslib.as_array(ptr, (n,)).copy() if n else np.zeros(0, dtype=np.uint32)
        fc = col(v.fint_col, int(fo[-1]))
        rc = col(v.rev_col, int(ro[-1]))
        return {"N": n, "Nx": nx, "Ni": v.num_interior, "fint_off": fo, "fint_col": fc, "rev_off": ro, "rev_col": rc}

    def core_index(self, closure_cap=(64, 64), block=(0, 0)):
        """plan core's record arrays as the engine builds them (ketogpu_core_index_build):
        per direction a dict with `records` (n x 4 uint32: node, deg, begin, pad),
        block_base, block_records and the closure / overflow counts"""
        cap = (C.c_uint32 * 2)(*closure_cap)
        blk = (C.c_uint32 * 2)(*block)
        h = C.c_void_p()
        L.check(self.L.ketogpu_core_index_build(self.h, cap, blk, C.byref(h)))
        try:
            out = []
            for d in (0, 1):
                v = L.CoreRecords()
                L.check(self.L.ketogpu_core_index_view(h, d, C.byref(v)))
                rec = (np.ctypeslib.as_array(v.records, (v.num_records * 4,)).reshape(-1, 4).copy()
                       if v.num_records else np.zeros((0, 4), dtype=np.uint32))
                out.append({"records": rec, "block_base": v.block_base, "block_records": v.block_records,
                            "overflow_rows": v.overflow_rows, "closure_nodes": v.closure_nodes,
                            "closure_entries": v.closure_entries})
            return out
        finally:
            self.L.ketogpu_core_index_free(h)

    def label_index(self, s_head_words=0, p_head_words=0):
        """plan label's 2-hop labels and head arrays as the engine builds them
        (ketogpu_label_index_build, labels.hpp): dict with the S and P word arrays, the head
        sizes and the counts"""
        h = C.c_void_p()
        L.check(self.L.ketogpu_label_index_build(self.h, s_head_words, p_head_words, C.byref(h)))
        try:
            v = L.LabelView()
            L.check(self.L.ketogpu_label_index_view(h, C.byref(v)))
            arr = lambda p, n: np.ctypeslib.as_array(p, (n,)).copy() if n else np.zeros(0, dtype=np.uint32)
            d = {k: getattr(v, k) for k, _ in v._fields_ if k not in ("s_words", "p_words")}
            d["S"], d["P"] = arr(v.s_words, v.num_s_words), arr(v.p_words, v.num_p_words)
            return d
        finally:
            self.L.ketogpu_label_index_free(h)

    def resolve(self, namespace, obj, relation, subject):
        """-> (root, target) node ids (KETOGPU_NODE_NONE when absent)"""
        req = L.CheckRequest(L.b(namespace), L.b(obj), L.b(relation), subject_struct(subject))
        r, t = C.c_uint32(), C.c_uint32()
        L.check(self.L.ketogpu_resolve(self.h, C.byref(req), C.byref(r), C.byref(t)))
        return r.value, t.value

    def resolve_batch(self, cols):
        """ketogpu_resolve_batch over request columns (persistence.request_columns) or a
        ready L.RequestBatch -> (roots, targets, status)"""
        rb = cols if isinstance(cols, L.RequestBatch) else L.request_batch(cols)
        n = rb.n
        roots = np.empty(max(n, 1), dtype=np.uint32)
        targets = np.empty(max(n, 1), dtype=np.uint32)
        status = np.empty(max(n, 1), dtype=np.int32)
        L.check(self.L.ketogpu_resolve_batch(self.h, C.byref(rb), roots.ctypes.data, targets.ctypes.data,
                                             status.ctypes.data))
        return roots[:n], targets[:n], status[:n]

    def resolve_many(self, requests):
        roots = np.empty(len(requests), dtype=np.uint32)
        targets = np.empty(len(requests), dtype=np.uint32)
        for i, (ns, obj, rel, subj) in enumerate(requests):
            roots[i], targets[i] = self.resolve(ns, obj, rel, subj)
        return roots, targets
