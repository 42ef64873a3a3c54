"""ctypes wrapper of the C oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  It loads oracle/build/libketo_oracle.so (built by `make -C oracle`)
and exposes the reference semantics restated in keto_oracle.c.
"""
import ctypes as C
import json
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libketo_oracle.so")
_lib = None

OK, ENOTFOUND, EINVAL, ENOMEM, ETIMEOUT = 0, -1, -2, -3, -4
SUBJECT_ID, SUBJECT_SET, SUBJECT_NIL = 0, 1, -1


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        vp, cp, i32, i64, u64p = C.c_void_p, C.c_char_p, C.c_int32, C.c_int64, C.POINTER(C.c_uint64)
        L.ko_store_new.restype = vp
        L.ko_store_free.argtypes = [vp]
        L.ko_add_namespace.argtypes = [vp, i32, cp]
        L.ko_set_page_size.argtypes = [vp, C.c_int]
        L.ko_set_nulls_last.argtypes = [vp, C.c_int]
        L.ko_add_row.argtypes = [vp, i32, cp, cp, cp, i32, cp, cp, i64]
        L.ko_add_rows_columnar.argtypes = [vp, C.c_size_t] + [vp] * 14
        L.ko_finalize.argtypes = [vp, C.c_int]
        L.ko_num_rows.argtypes = [vp]
        L.ko_num_rows.restype = C.c_size_t
        L.ko_check.argtypes = [vp, cp, cp, cp, C.c_int, cp, cp, cp, cp, C.POINTER(C.c_int)]
        L.ko_check_batch.argtypes = [vp, C.c_size_t, vp, vp, vp, vp, vp, vp, vp, vp, C.c_int, vp, vp]
        L.ko_check_batch_budget.argtypes = [vp, C.c_size_t, vp, vp, vp, vp, vp, vp, vp, vp, C.c_int, C.c_double,
                                            vp, vp]
        L.ko_expand.argtypes = [vp, C.c_int, cp, cp, cp, cp, C.c_int, C.POINTER(C.c_void_p)]
        L.ko_get_page.argtypes = [vp, cp, cp, cp, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_int)]
        L.ko_free.argtypes = [vp]
        _lib = L
    return _lib


def _b(s):
    return None if s is None else s.encode("utf-8")


class OracleError(Exception):
    def __init__(self, code):
        super().__init__({ENOTFOUND: "not_found", EINVAL: "invalid", ENOMEM: "nomem"}.get(code, str(code)))
        self.code = code
        self.kind = {ENOTFOUND: "not_found", EINVAL: "invalid"}.get(code, "error")


def subject_args(d):
    """subject of a fixture dict -> (kind, id, ns, obj, rel)"""
    if d.get("subject_id") is not None:
        return SUBJECT_ID, d["subject_id"], None, None, None
    if d.get("subject_set") is not None:
        s = d["subject_set"]
        return SUBJECT_SET, None, s["namespace"], s["object"], s["relation"]
    return SUBJECT_NIL, None, None, None, None


class Store:
    """keto_relation_tuples + namespace config, read through the reference's queries."""

    def __init__(self, namespaces, page_size=100, order="sqlite"):
        """order: the backend whose ORDER BY is restated — "sqlite" (NULLs first, the
        reference's tests) or "postgres" (NULLs last, "C" collation)"""
        self.L = lib()
        self.h = self.L.ko_store_new()
        self.namespaces = list(namespaces)  # [(name, id)] in config order
        for name, nid in self.namespaces:
            self.L.ko_add_namespace(self.h, nid, _b(name))
        self.L.ko_set_page_size(self.h, page_size)
        self.L.ko_set_nulls_last(self.h, {"sqlite": 0, "postgres": 1}[order])
        self._ct = 0

    def __del__(self):
        if getattr(self, "h", None):
            self.L.ko_store_free(self.h)
            self.h = None

    def ns_id(self, name):
        for n, i in self.namespaces:  # GetNamespaceByName: first match
            if n == name:
                return i
        raise KeyError(name)

    def add_row(self, namespace_id, obj, rel, subject_id=None, ss_ns_id=0, ss_obj=None, ss_rel=None, commit_time=None):
        if commit_time is None:
            commit_time = self._ct
        self._ct += 1
        rc = self.L.ko_add_row(self.h, namespace_id, _b(obj), _b(rel), _b(subject_id), ss_ns_id, _b(ss_obj),
                               _b(ss_rel), commit_time)
        if rc:
            raise OracleError(rc)

    def add_tuple(self, t):
        """InsertRelationTuple: namespace names resolved to ids (relationtuples.go:82-126)"""
        kind, sid, sns, sobj, srel = subject_args(t)
        if kind == SUBJECT_ID:
            self.add_row(self.ns_id(t["namespace"]), t["object"], t["relation"], subject_id=sid)
        else:
            self.add_row(self.ns_id(t["namespace"]), t["object"], t["relation"], ss_ns_id=self.ns_id(sns),
                         ss_obj=sobj, ss_rel=srel)

    def add_columnar(self, cols):
        """cols: dict of numpy arrays in the ketogpu_row_batch layout"""
        n = len(cols["namespace_id"])
        p = lambda a: None if a is None else a.ctypes.data
        rc = self.L.ko_add_rows_columnar(
            self.h, n, p(cols["namespace_id"]), p(cols["object_data"]), p(cols["object_off"]),
            p(cols["relation_data"]), p(cols["relation_off"]), p(cols["subject_kind"]),
            p(cols["subject_id_data"]), p(cols["subject_id_off"]), p(cols["ss_namespace_id"]),
            p(cols["ss_object_data"]), p(cols["ss_object_off"]), p(cols["ss_relation_data"]),
            p(cols["ss_relation_off"]), p(cols.get("commit_time")))
        if rc:
            raise OracleError(rc)

    def finalize(self, presorted=False):
        rc = self.L.ko_finalize(self.h, 1 if presorted else 0)
        if rc:
            raise OracleError(rc)
        return self

    def check(self, ns, obj, rel, subject):
        kind, sid, sns, sobj, srel = subject_args(subject)
        out = C.c_int(0)
        rc = self.L.ko_check(self.h, _b(ns), _b(obj), _b(rel), kind, _b(sid), _b(sns), _b(sobj), _b(srel),
                             C.byref(out))
        if rc:
            raise OracleError(rc)
        return bool(out.value)

    def check_batch(self, reqs, nthreads=1):
        """reqs: list of (ns, obj, rel, subject dict) -> list of bools"""
        import numpy as np
        n = len(reqs)
        keep = []

        def arr(vals):
            a = (C.c_char_p * n)(*[_b(v) for v in vals])
            keep.append(a)
            return a

        subj = [subject_args(r[3]) for r in reqs]
        kinds = (C.c_int * n)(*[s[0] for s in subj])
        allowed = np.zeros(n, dtype=np.uint8)
        status = np.zeros(n, dtype=np.int32)
        self.L.ko_check_batch(self.h, n, arr([r[0] for r in reqs]), arr([r[1] for r in reqs]),
                              arr([r[2] for r in reqs]), kinds, arr([s[1] for s in subj]), arr([s[2] for s in subj]),
                              arr([s[3] for s in subj]), arr([s[4] for s in subj]), nthreads,
                              allowed.ctypes.data, status.ctypes.data)
        if status.any():
            raise OracleError(int(status[status != 0][0]))
        return allowed.astype(bool)

    def check_batch_budget(self, reqs, nthreads=1, seconds=60.0):
        """check_batch with a time budget per request -> (allowed, completed mask): a
        request whose DFS runs out of time is reported, not answered"""
        import numpy as np
        n = len(reqs)
        keep = []

        def arr(vals):
            a = (C.c_char_p * max(n, 1))(*[_b(v) for v in vals])
            keep.append(a)
            return a

        subj = [subject_args(r[3]) for r in reqs]
        kinds = (C.c_int * max(n, 1))(*[s[0] for s in subj])
        allowed = np.zeros(max(n, 1), dtype=np.uint8)
        status = np.zeros(max(n, 1), dtype=np.int32)
        self.L.ko_check_batch_budget(self.h, n, arr([r[0] for r in reqs]), arr([r[1] for r in reqs]),
                                     arr([r[2] for r in reqs]), kinds, arr([s[1] for s in subj]),
                                     arr([s[2] for s in subj]), arr([s[3] for s in subj]), arr([s[4] for s in subj]),
                                     nthreads, seconds, allowed.ctypes.data, status.ctypes.data)
        bad = status[:n][(status[:n] != OK) & (status[:n] != ETIMEOUT)]
        if len(bad):
            raise OracleError(int(bad[0]))
        return allowed[:n].astype(bool), status[:n] == OK

    def expand(self, subject, max_depth):
        kind, sid, sns, sobj, srel = subject_args(subject)
        out = C.c_void_p()
        rc = self.L.ko_expand(self.h, kind, _b(sid), _b(sns), _b(sobj), _b(srel), max_depth, C.byref(out))
        if rc:
            raise OracleError(rc)
        s = C.string_at(out.value).decode("utf-8")
        self.L.ko_free(out)
        return json.loads(s)

    def get_page(self, ns, obj, rel, page=1):
        out, nxt = C.c_void_p(), C.c_int(0)
        rc = self.L.ko_get_page(self.h, _b(ns), _b(obj), _b(rel), page, C.byref(out), C.byref(nxt))
        if rc:
            raise OracleError(rc)
        s = C.string_at(out.value).decode("utf-8")
        self.L.ko_free(out)
        return json.loads(s), bool(nxt.value)


def store_from_case(case):
    st = Store([(n["name"], n["id"]) for n in case["namespaces"]], case.get("page_size", 100))
    for t in case["tuples"]:
        st.add_tuple(t)
    return st.finalize()


# ----------------------------------------------------------------- keto_sql (B2)
_SQL_PATH = os.path.join(_HERE, "build", "libketo_sql.so")
_sql = None


def sql_lib():
    global _sql
    if _sql is None:
        if not os.path.exists(_SQL_PATH):
            build()
        L = C.CDLL(_SQL_PATH)
        vp = C.c_void_p
        L.ks_db_create.restype = vp
        L.ks_db_create.argtypes = [C.c_char_p, C.c_int]
        L.ks_db_add_namespace.argtypes = [vp, C.c_int32, C.c_char_p]
        L.ks_db_add_rows_columnar.argtypes = [vp, C.c_size_t] + [vp] * 14
        L.ks_db_finish.argtypes = [vp]
        L.ks_db_free.argtypes = [vp]
        L.ks_check_batch.argtypes = [vp, C.c_size_t] + [vp] * 8 + [C.c_int, C.c_double, vp, vp,
                                                                    C.POINTER(C.c_size_t), C.POINTER(C.c_longlong)]
        _sql = L
    return _sql


SKIPPED = -9


class SqlStore:
    """keto_relation_tuples in a real SQLite file read through the reference's queries
    (oracle/keto_sql.c: COUNT + ORDER BY/LIMIT/OFFSET per page per expansion), one
    connection per worker thread.  BASELINE.md B2."""

    def __init__(self, namespaces, page_size=100, path=None):
        self.L = sql_lib()
        if path is None:
            d = "/dev/shm" if os.path.isdir("/dev/shm") else "/tmp"
            path = os.path.join(d, f"keto_sql_{os.getpid()}_{id(self)}.db")
        self.path = path
        self.h = self.L.ks_db_create(_b(path), page_size)
        if not self.h:
            raise OracleError(EINVAL)
        for name, nid in namespaces:
            self.L.ks_db_add_namespace(self.h, nid, _b(name))

    def add_columnar(self, cols):
        p = lambda a: None if a is None else a.ctypes.data
        rc = self.L.ks_db_add_rows_columnar(
            self.h, len(cols["namespace_id"]), p(cols["namespace_id"]), p(cols["object_data"]), p(cols["object_off"]),
            p(cols["relation_data"]), p(cols["relation_off"]), p(cols["subject_kind"]), p(cols["subject_id_data"]),
            p(cols["subject_id_off"]), p(cols["ss_namespace_id"]), p(cols["ss_object_data"]),
            p(cols["ss_object_off"]), p(cols["ss_relation_data"]), p(cols["ss_relation_off"]),
            p(cols.get("commit_time")))
        if rc:
            raise OracleError(rc)

    def finish(self):
        rc = self.L.ks_db_finish(self.h)
        if rc:
            raise OracleError(rc)
        return self

    def check_batch(self, reqs, nthreads=1, seconds=0.0):
        """reqs: [(ns, obj, rel, subject dict)] -> (allowed bool array, answered mask, SQL
        statements issued); requests past the time budget are not answered"""
        import numpy as np
        n = len(reqs)
        keep = []

        def arr(vals):
            a = (C.c_char_p * n)(*[_b(v if v is not None else "") for v in vals])
            keep.append(a)
            return a

        subj = [subject_args(r[3]) for r in reqs]
        kinds = (C.c_int * n)(*[s[0] for s in subj])
        allowed = np.zeros(n, dtype=np.uint8)
        status = np.zeros(n, dtype=np.int32)
        done, queries = C.c_size_t(), C.c_longlong()
        self.L.ks_check_batch(self.h, n, arr([r[0] for r in reqs]), arr([r[1] for r in reqs]),
                              arr([r[2] for r in reqs]), kinds, arr([s[1] for s in subj]), arr([s[2] for s in subj]),
                              arr([s[3] for s in subj]), arr([s[4] for s in subj]), nthreads, seconds,
                              allowed.ctypes.data, status.ctypes.data, C.byref(done), C.byref(queries))
        bad = status[(status != 0) & (status != SKIPPED)]
        if len(bad):
            raise OracleError(int(bad[0]))
        return allowed.astype(bool), status == 0, int(queries.value)

    def close(self):
        if getattr(self, "h", None):
            self.L.ks_db_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


# ------------------------------------------------------------ r2_check (scale pins)
_R2_PATH = os.path.join(_HERE, "build", "libr2_check.so")
_r2 = None


def r2_lib():
    global _r2
    if _r2 is None:
        if not os.path.exists(_R2_PATH):
            build()
        L = C.CDLL(_R2_PATH)
        vp = C.c_void_p
        L.kr_new.restype = vp
        L.kr_new.argtypes = [vp, vp, C.c_size_t]
        L.kr_add_requests.argtypes = [vp, C.c_size_t] + [vp] * 8
        L.kr_add_rows_columnar.argtypes = [vp, C.c_size_t] + [vp] * 13
        L.kr_finish.argtypes = [vp]
        L.kr_check.argtypes = [vp, C.c_int, vp, vp, C.POINTER(C.c_uint64), vp]
        L.kr_stats.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.kr_error.restype = C.c_char_p
        L.kr_error.argtypes = [vp]
        L.kr_free.argtypes = [vp]
        _r2 = L
    return _r2


class R2Checker:
    """allowed(r, t) <=> r in P(t) or P(t) ∩ X(r) != {} over the raw rows (oracle/r2_check.c):
    an independent check for graphs the reference DFS cannot finish.  Requests first, then
    the row stream, then check()."""

    def __init__(self, namespaces, reqs):
        self.L = r2_lib()
        ids = (C.c_int32 * max(len(namespaces), 1))(*[i for _, i in namespaces])
        names = (C.c_char_p * max(len(namespaces), 1))(*[_b(n) for n, _ in namespaces])
        self.h = self.L.kr_new(ids, names, len(namespaces))
        n = self.n = len(reqs)
        keep = self._keep = []

        def arr(vals):
            a = (C.c_char_p * max(n, 1))(*[_b(v if v is not None else "") for v in vals])
            keep.append(a)
            return a
        subj = [subject_args(r[3]) for r in reqs]
        kinds = (C.c_int * max(n, 1))(*[s[0] for s in subj])
        keep.append(kinds)
        self.L.kr_add_requests(self.h, n, arr([r[0] for r in reqs]), arr([r[1] for r in reqs]),
                               arr([r[2] for r in reqs]), kinds, arr([s[1] for s in subj]), arr([s[2] for s in subj]),
                               arr([s[3] for s in subj]), arr([s[4] for s in subj]))

    def add_columnar(self, cols):
        p = lambda a: None if a is None else a.ctypes.data
        rc = self.L.kr_add_rows_columnar(
            self.h, len(cols["namespace_id"]), p(cols["namespace_id"]), p(cols["object_data"]), p(cols["object_off"]),
            p(cols["relation_data"]), p(cols["relation_off"]), p(cols["subject_kind"]), p(cols["subject_id_data"]),
            p(cols["subject_id_off"]), p(cols["ss_namespace_id"]), p(cols["ss_object_data"]),
            p(cols["ss_object_off"]), p(cols["ss_relation_data"]), p(cols["ss_relation_off"]))
        if rc:
            raise OracleError(rc) from RuntimeError(self.L.kr_error(self.h).decode())
        return self

    def check(self, nthreads=1):
        """-> (allowed bool array, in-scope mask)"""
        import numpy as np
        rc = self.L.kr_finish(self.h)
        if rc:
            raise OracleError(rc)
        allowed = np.zeros(max(self.n, 1), dtype=np.uint8)
        status = np.zeros(max(self.n, 1), dtype=np.int32)
        visits = C.c_uint64()
        closure = np.zeros(max(self.n, 1), dtype=np.uint64)
        self.L.kr_check(self.h, nthreads, allowed.ctypes.data, status.ctypes.data, C.byref(visits), closure.ctypes.data)
        self.edge_visits = visits.value
        self.closure_size = closure[:self.n]  # per request: the interior nodes its root reaches
        return allowed[:self.n].astype(bool), status[:self.n] == 0

    def stats(self):
        nodes, edges = C.c_uint64(), C.c_uint64()
        self.L.kr_stats(self.h, C.byref(nodes), C.byref(edges))
        return {"set_nodes": nodes.value, "set_edges": edges.value}

    def close(self):
        if getattr(self, "h", None):
            self.L.kr_free(self.h)
            self.h = None

    def __del__(self):
        self.close()
