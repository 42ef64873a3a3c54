"""Synthetic workloads of BASELINE.json (driver of keto_amd/csrc/synth.cpp).

Config #2 — synthetic RBAC: 10M users, 100k nested groups,
50M tuples, 1M checks docs:d#viewer@u (half constructed positives), seed 0x4B45544F.
Config #3 — drive-like folders (parent#viewer subject sets, depth 10, 500M tuples).
Config #4 — power-law social/group graph (1B tuples).  Full sizes are the defaults of
rbac() / folders() / social(); tests and quick runs pass smaller sizes.
Rows come out in the reference's ORDER BY order (SQLite semantics), i.e. exactly what
the snapshot loader would read from the database.
"""
import ctypes as C
import os

import numpy as np

from . import _lib as L

HERE = os.path.dirname(os.path.abspath(__file__))
SEED = 0x4B45544F
_slib = None


class Params(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("users", "groups", "docs", "tuples", "checks", "seed")] + [
        ("zipf_s", C.c_double), ("member_mean", C.c_double), ("check_seed", C.c_uint64)]


class FolderParams(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("users", "groups", "folders", "tuples", "checks", "seed")] + [
        ("member_mean", C.c_double), ("group_frac", C.c_double), ("depth", C.c_uint64), ("check_seed", C.c_uint64)]


class SocialParams(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("users", "groups", "tuples", "checks", "seed")] + [
        ("zipf_s", C.c_double), ("member_mean", C.c_double), ("nest_per_group", C.c_double),
        ("check_seed", C.c_uint64)]


class C5Params(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("users", "groups", "docs", "tuples", "seed")] + [
        ("zipf_s", C.c_double), ("member_mean", C.c_double)]


class View(C.Structure):
    _fields_ = [("n", C.c_uint64)] + [(n, C.c_void_p) for n in (
        "namespace_id", "object_data", "object_off", "relation_data", "relation_off", "subject_kind",
        "subject_id_data", "subject_id_off", "ss_namespace_id", "ss_object_data", "ss_object_off",
        "ss_relation_data", "ss_relation_off")] + [("n_checks", C.c_uint64)] + [(n, C.c_void_p) for n in (
        "chk_doc", "chk_user", "chk_pos", "rq_ns_data", "rq_ns_off", "rq_obj_data", "rq_obj_off", "rq_rel_data",
        "rq_rel_off", "rq_sid_data", "rq_sid_off")] + [(n, C.c_uint64) for n in ("n_parent", "n_member", "n_grant")]


def slib():
    global _slib
    if _slib is None:
        path = os.path.join(HERE, "libketosynth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `python -m keto_amd.build`")
        _slib = C.CDLL(path)
        _slib.ks_rbac_generate.restype = C.c_void_p
        _slib.ks_rbac_generate.argtypes = [C.POINTER(Params)]
        _slib.ks_folders_generate.restype = C.c_void_p
        _slib.ks_folders_generate.argtypes = [C.POINTER(FolderParams)]
        _slib.ks_social_generate.restype = C.c_void_p
        _slib.ks_social_generate.argtypes = [C.POINTER(SocialParams)]
        _slib.ks_rbac_view_get.argtypes = [C.c_void_p, C.POINTER(View)]
        _slib.ks_c5_new.restype = C.c_void_p
        _slib.ks_c5_new.argtypes = [C.POINTER(C5Params)]
        _slib.ks_c5_rewind.argtypes = [C.c_void_p]
        _slib.ks_c5_next.restype = C.c_uint64
        _slib.ks_c5_next.argtypes = [C.c_void_p, C.c_uint64]
        _slib.ks_c5_checks.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64]
        _slib.ks_c5_buffers.restype = C.c_void_p
        _slib.ks_c5_buffers.argtypes = [C.c_void_p]
        _slib.ks_c5_free.argtypes = [C.c_void_p]
        _slib.ks_rbac_free.argtypes = [C.c_void_p]
    return _slib


def _arr(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    ct = np.ctypeslib.as_ctypes_type(np.dtype(dtype))
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), (n,))


class Workload:
    """rows (columnar, ORDER BY order) + check requests; arrays view C++ memory.
    A request i is (ns, f"{prefix}{chk_doc[i]}", relation) @ u{chk_user[i]}."""

    def __init__(self, params, kind="rbac"):
        self.params = params
        self.kind = kind
        gen, self.namespaces, self.request_shape = {
            "rbac": (slib().ks_rbac_generate, [("groups", 1), ("docs", 2)], ("docs", "d", "viewer")),
            "folders": (slib().ks_folders_generate, [("groups", 1), ("folders", 2)], ("folders", "f", "viewer")),
            "social": (slib().ks_social_generate, [("groups", 1)], ("groups", "g", "member")),
        }[kind]
        self.h = gen(C.byref(params))
        v = View()
        slib().ks_rbac_view_get(self.h, C.byref(v))
        self.v = v
        n = v.n
        off = lambda p: _arr(p, n + 1, np.uint64)
        data = lambda p, o: _arr(p, int(o[-1]), np.uint8) if int(o[-1]) else np.zeros(1, np.uint8)
        cols = {"namespace_id": _arr(v.namespace_id, n, np.int32), "subject_kind": _arr(v.subject_kind, n, np.uint8),
                "ss_namespace_id": _arr(v.ss_namespace_id, n, np.int32)}
        for c in ("object", "relation", "subject_id", "ss_object", "ss_relation"):
            o = off(getattr(v, c + "_off"))
            cols[c + "_off"] = o
            cols[c + "_data"] = data(getattr(v, c + "_data"), o)
        cols["commit_time"] = None
        self.columns = cols
        m = v.n_checks
        self.n_checks = m
        self.chk_doc = _arr(v.chk_doc, m, np.uint32)
        self.chk_user = _arr(v.chk_user, m, np.uint32)
        self.chk_pos = _arr(v.chk_pos, m, np.uint8)
        self.counts = {"parent": v.n_parent, "member": v.n_member, "grant": v.n_grant, "tuples": n}

    def __del__(self):
        if getattr(self, "h", None) and _slib is not None:
            _slib.ks_rbac_free(self.h)
            self.h = None

    def request_batch(self):
        v, m = self.v, self.n_checks
        return L.RequestBatch(m, v.rq_ns_data, v.rq_ns_off, v.rq_obj_data, v.rq_obj_off, v.rq_rel_data, v.rq_rel_off,
                              None, v.rq_sid_data, v.rq_sid_off, None, None, None, None, None, None)

    def resolve(self, snap):
        """host resolution of all checks -> (roots, targets) node ids"""
        m = self.n_checks
        roots = np.empty(m, dtype=np.uint32)
        targets = np.empty(m, dtype=np.uint32)
        status = np.empty(m, dtype=np.int32)
        rb = self.request_batch()
        L.check(L.lib().ketogpu_resolve_batch(snap.h, C.byref(rb), roots.ctypes.data, targets.ctypes.data,
                                              status.ctypes.data))
        assert not status.any()
        return roots, targets

    def requests(self, idx):
        """(ns, obj, rel, subject dict) for the oracle"""
        ns, prefix, rel = self.request_shape
        return [(ns, f"{prefix}{int(self.chk_doc[i])}", rel, {"subject_id": f"u{int(self.chk_user[i])}"})
                for i in idx]


def rbac(users=10_000_000, groups=100_000, docs=2_000_000, tuples=50_000_000, checks=1_000_000, seed=SEED,
         zipf_s=1.1, member_mean=3.0, check_seed=0):
    """check_seed = 0: checks drawn from the graph's own random stream"""
    return Workload(Params(users, groups, docs, tuples, checks, seed, zipf_s, member_mean, check_seed))


def folders(users=10_000_000, groups=100_000, folders=20_000_000, tuples=500_000_000, checks=1_000_000, seed=SEED,
            member_mean=3.0, group_frac=0.1, depth=10, check_seed=0):
    """config #3: drive-like folder hierarchy (parent#viewer subject sets, depth 10)"""
    return Workload(FolderParams(users, groups, folders, tuples, checks, seed, member_mean, group_frac, depth,
                                 check_seed), "folders")


def social(users=100_000_000, groups=10_000_000, tuples=1_000_000_000, checks=1_000_000, seed=SEED, zipf_s=1.0,
           member_mean=8.0, nest_per_group=1.0, check_seed=0):
    """config #4: power-law social/group graph (Zipf popularity, acyclic nesting)"""
    return Workload(SocialParams(users, groups, tuples, checks, seed, zipf_s, member_mean, nest_per_group,
                                 check_seed), "social")


def _columns(v, n):
    off = lambda p: _arr(p, n + 1, np.uint64)
    data = lambda p, o: _arr(p, int(o[-1]), np.uint8) if int(o[-1]) else np.zeros(1, np.uint8)
    cols = {"namespace_id": _arr(v.namespace_id, n, np.int32), "subject_kind": _arr(v.subject_kind, n, np.uint8),
            "ss_namespace_id": _arr(v.ss_namespace_id, n, np.int32)}
    for c in ("object", "relation", "subject_id", "ss_object", "ss_relation"):
        o = off(getattr(v, c + "_off"))
        cols[c + "_off"] = o
        cols[c + "_data"] = data(getattr(v, c + "_data"), o)
    cols["commit_time"] = None
    return cols


class StreamWorkload:
    """config #5: the RBAC shape at billions of tuples, defined node by node and streamed in
    ORDER BY order (keto_amd/csrc/synth.cpp ks_c5_*): `batches()` is the one ordered read
    every rank of the partitioned loader takes; no process holds all rows.  Requests as
    Workload's (docs:d#viewer@u, half constructed positives)."""

    namespaces = [("groups", 1), ("docs", 2)]
    request_shape = ("docs", "d", "viewer")
    kind = "config5"

    def __init__(self, params, checks, check_seed=0):
        self.params = params
        self.h = slib().ks_c5_new(C.byref(params))
        slib().ks_c5_checks(self.h, checks, check_seed)
        v = View()
        slib().ks_rbac_view_get(slib().ks_c5_buffers(self.h), C.byref(v))
        self.n_checks = v.n_checks
        self.chk_doc = _arr(v.chk_doc, v.n_checks, np.uint32).copy()
        self.chk_user = _arr(v.chk_user, v.n_checks, np.uint32).copy()
        self.chk_pos = _arr(v.chk_pos, v.n_checks, np.uint8).copy()
        self._rq = v  # request columns stay valid: batches only rewrite the row columns

    def batches(self, batch_rows=1 << 20):
        """the ordered row stream, as column dicts valid until the next batch"""
        lib = slib()
        lib.ks_c5_rewind(self.h)
        done = 0
        while True:
            n = lib.ks_c5_next(self.h, batch_rows)
            if not n:
                return
            v = View()
            lib.ks_rbac_view_get(lib.ks_c5_buffers(self.h), C.byref(v))
            cols = _columns(v, n)
            cols["commit_time"] = np.arange(done, done + n, dtype=np.int64)  # insertion order across batches
            done += n
            yield cols

    def request_batch(self):
        v, m = self._rq, self.n_checks
        return L.RequestBatch(m, v.rq_ns_data, v.rq_ns_off, v.rq_obj_data, v.rq_obj_off, v.rq_rel_data, v.rq_rel_off,
                              None, v.rq_sid_data, v.rq_sid_off, None, None, None, None, None, None)

    requests = Workload.requests

    def __del__(self):
        if getattr(self, "h", None) and _slib is not None:
            _slib.ks_c5_free(self.h)
            self.h = None


def config5(users=500_000_000, groups=10_000_000, docs=200_000_000, tuples=5_000_000_000, checks=1_000_000,
            seed=SEED, zipf_s=1.1, member_mean=3.0, check_seed=0):
    """config #5 (BASELINE.json configs[4]): the RBAC shape at 5B tuples, streamed"""
    return StreamWorkload(C5Params(users, groups, docs, tuples, seed, zipf_s, member_mean), checks, check_seed)
