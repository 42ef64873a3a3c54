"""check.Engine — SubjectIsAllowed on the MI355X engine.

Mirrors internal/check/engine.go: `Engine.SubjectIsAllowed(tuple)` keeps the
reference's name, argument and error behaviour (unknown namespace -> False,
engine.go:75-77; nil subject -> ErrNilSubject, a documented divergence: the
reference dereferences it).  `check_many` is the batch form every call goes through:
requests are resolved on the host and traversed on the GPU (device_engine.hip).
"""
import ctypes as C

import numpy as np

from . import _lib as L
from .relationtuple import InternalRelationTuple, NilSubject
from .snapshot import Snapshot, subject_struct


class Engine:
    def __init__(self, snapshot: Snapshot, device=0, max_words_per_round=0, state_budget_bytes=0):
        self.L = L.lib()
        self.snapshot = snapshot  # keeps the snapshot alive
        opts = L.EngineOpts(device, max_words_per_round, state_budget_bytes)
        h = C.c_void_p()
        L.check(self.L.ketogpu_engine_new(snapshot.h, C.byref(opts), C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.L.ketogpu_engine_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    # ------------------------------------------------------------ reference API
    def SubjectIsAllowed(self, r: InternalRelationTuple) -> bool:
        return self.check_many([r])[0]

    subject_is_allowed = SubjectIsAllowed

    def check_many(self, tuples):
        """list of InternalRelationTuple -> list of bool (raises NilSubject like the API would 400)"""
        n = len(tuples)
        reqs = (L.CheckRequest * max(n, 1))()
        for i, t in enumerate(tuples):
            reqs[i] = L.CheckRequest(L.b(t.namespace), L.b(t.object), L.b(t.relation), subject_struct(t.subject))
        allowed = np.zeros(max(n, 1), dtype=np.uint8)
        status = np.zeros(max(n, 1), dtype=np.int32)
        L.check(self.L.ketogpu_check(self.h, reqs, n, allowed.ctypes.data, status.ctypes.data))
        if (status[:n] == L.EINVAL).any():
            raise NilSubject("subject is not allowed to be nil")
        return [bool(a) for a in allowed[:n]]

    # ------------------------------------------------------------ id-level API
    def check_ids(self, roots, targets, with_flags=False):
        roots = np.ascontiguousarray(roots, dtype=np.uint32)
        targets = np.ascontiguousarray(targets, dtype=np.uint32)
        n = len(roots)
        words = max((n + 63) // 64, 1)
        ab = np.zeros(words, dtype=np.uint64)
        fb = np.zeros(words, dtype=np.uint64)
        L.check(self.L.ketogpu_check_ids(self.h, roots.ctypes.data, targets.ctypes.data, n, ab.ctypes.data,
                                         fb.ctypes.data))
        allowed = unpack_bits(ab, n)
        return (allowed, unpack_bits(fb, n)) if with_flags else allowed

    def upload(self, roots, targets):
        return DeviceQueries(self, roots, targets)

    def last_stats(self):
        st = L.RunStats()
        L.check(self.L.ketogpu_engine_last_stats(self.h, C.byref(st)))
        return st.as_dict()


def unpack_bits(words, n):
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")
    return bits[:n].astype(bool)


class DeviceQueries:
    """a request batch resident in HBM (ketogpu_queries_*)"""

    def __init__(self, engine: Engine, roots, targets):
        self.e = engine
        self.roots = np.ascontiguousarray(roots, dtype=np.uint32)
        self.targets = np.ascontiguousarray(targets, dtype=np.uint32)
        self.n = len(self.roots)
        h = C.c_void_p()
        L.check(engine.L.ketogpu_queries_upload(engine.h, self.roots.ctypes.data, self.targets.ctypes.data, self.n,
                                                C.byref(h)))
        self.h = h

    def run(self):
        L.check(self.e.L.ketogpu_queries_run(self.e.h, self.h))

    def download(self, with_flags=False):
        words = max((self.n + 63) // 64, 1)
        ab = np.zeros(words, dtype=np.uint64)
        fb = np.zeros(words, dtype=np.uint64)
        L.check(self.e.L.ketogpu_queries_download(self.e.h, self.h, ab.ctypes.data, fb.ctypes.data))
        return (unpack_bits(ab, self.n), unpack_bits(fb, self.n)) if with_flags else unpack_bits(ab, self.n)

    def close(self):
        if getattr(self, "h", None):
            self.e.L.ketogpu_queries_free(self.h)
            self.h = None

    def __del__(self):
        self.close()
