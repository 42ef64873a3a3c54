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
        self.owned = True

    @classmethod
    def borrowed(cls, handle, snapshot, owner):
        """a view of an engine owned by something else (MultiEngine.engine(i))"""
        e = cls.__new__(cls)
        e.L, e.snapshot, e.h, e.owned, e._owner = L.lib(), snapshot, C.c_void_p(handle), False, owner
        return e

    def close(self):
        if getattr(self, "h", None):
            if getattr(self, "owned", True):
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

    def check_batch(self, tuples):
        """check_many through the throughput path: ketogpu_resolve_batch on the host, one
        ketogpu_check_ids over the resolved ids (H2D, traversal, D2H).  Requests that need
        the sequential semantics — a wildcard root without a snapshot node (status
        ENOTFOUND) or a traversal that touched a shared String() key (R4 flag) — are
        re-answered by ketogpu_check.  Nil subjects raise NilSubject like check_many."""
        from .persistence import request_columns
        n = len(tuples)
        if not n:
            return []
        cols = request_columns([(t.namespace, t.object, t.relation, t.subject) for t in tuples])
        roots, targets, status = self.snapshot.resolve_batch(cols)
        if (status == L.EINVAL).any():
            raise NilSubject("subject is not allowed to be nil")
        allowed, flagged = self.check_ids(roots, targets, with_flags=True)
        redo = np.flatnonzero(flagged | (status == L.ENOTFOUND))
        out = [bool(a) for a in allowed]
        if len(redo):
            for i, a in zip(redo, self.check_many([tuples[i] for i in redo])):
                out[i] = a
        return out

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

    def check_ids_raw(self, roots_ptr, targets_ptr, n, allowed_ptr, flagged_ptr=None):
        """the C call on caller-owned (e.g. pinned) buffers, no conversions (benchmarks)"""
        L.check(self.L.ketogpu_check_ids(self.h, roots_ptr, targets_ptr, n, allowed_ptr, flagged_ptr))

    def upload(self, roots, targets):
        return DeviceQueries(self, roots, targets)

    def check_graph(self):
        """test hook (ketogpu_engine_check_graph): device rows and records that differ from
        the snapshot's host rows"""
        bad = C.c_uint64()
        L.check(self.L.ketogpu_engine_check_graph(self.h, C.byref(bad)))
        self.check_graph_first = self.L.ketogpu_last_error().decode("utf-8", "replace") if bad.value else ""
        return bad.value

    def label_heads(self, side):
        """test hook (ketogpu_engine_label_heads): plan label's S (side 0) or P (side 1) head
        array as built on the device -> (uint32 array or None, head words)"""
        words, hw = C.c_uint64(), C.c_uint32()
        L.check(self.L.ketogpu_engine_label_heads(self.h, side, None, 0, C.byref(words), C.byref(hw)))
        if not words.value:
            return None, 0
        out = np.empty(words.value, dtype=np.uint32)
        L.check(self.L.ketogpu_engine_label_heads(self.h, side, out.ctypes.data, words.value, C.byref(words),
                                                  C.byref(hw)))
        return out, hw.value

    def sync(self):
        """upload the device rows an in-place write patched (ketogpu_engine_sync; every
        check call does it first) -> (host ms, rows uploaded)"""
        ms, rows = C.c_double(), C.c_uint64()
        L.check(self.L.ketogpu_engine_sync(self.h, C.byref(ms), C.byref(rows)))
        return ms.value, rows.value

    def last_stats(self):
        st = L.RunStats()
        L.check(self.L.ketogpu_engine_last_stats(self.h, C.byref(st)))
        return st.as_dict()

    def wait(self):
        """waits for the calls enqueued on this engine (DeviceQueries.run(pipelined=True))"""
        L.check(self.L.ketogpu_engine_wait(self.h))

    def set_events(self, every_kernel):
        """host-to-host batches: a timing event between the call's kernels (main_ms = the
        first stage's own time) or only around the call (default)"""
        L.check(self.L.ketogpu_engine_set_events(self.h, 1 if every_kernel else 0))


class PinnedBuffer:
    """pinned host memory (ketogpu_host_alloc) viewed as a numpy array: a request batch
    written here is copied to HBM by DMA at full PCIe rate by check_ids"""

    def __init__(self, n, dtype=np.uint32):
        self.L = L.lib()
        dt = np.dtype(dtype)
        p = C.c_void_p()
        L.check(self.L.ketogpu_host_alloc(max(n, 1) * dt.itemsize, C.byref(p)))
        self.p = p
        buf = (C.c_char * (max(n, 1) * dt.itemsize)).from_address(p.value)
        self.array = np.frombuffer(buf, dtype=dt)[:n]

    def close(self):
        if getattr(self, "p", None):
            self.array = None
            self.L.ketogpu_host_free(self.p)
            self.p = None

    def __del__(self):
        self.close()


def pinned(values, dtype=np.uint32):
    """a PinnedBuffer holding a copy of `values` (keep the buffer alive while it is used)"""
    values = np.asarray(values, dtype=dtype)
    b = PinnedBuffer(len(values), dtype)
    b.array[:] = values
    return b


class MultiEngine:
    """One engine per device over the same snapshot (ketogpu_multi_*): check_ids splits a
    batch into contiguous 64-request-word ranges, one per device, run concurrently; the
    answers are exactly Engine.check_ids's (SURVEY.md 8(e) "Replicated")."""

    def __init__(self, snapshot: Snapshot, devices, max_words_per_round=0, state_budget_bytes=0):
        self.L = L.lib()
        self.snapshot = snapshot
        self.devices = [int(d) for d in devices]
        dev = (C.c_int32 * max(len(self.devices), 1))(*self.devices)
        opts = L.EngineOpts(0, max_words_per_round, state_budget_bytes)
        h = C.c_void_p()
        L.check(self.L.ketogpu_multi_new(snapshot.h, dev, len(self.devices), C.byref(opts), C.byref(h)))
        self.h = h

    @staticmethod
    def ranges(n, parts):
        lib = L.lib()
        out = []
        for i in range(parts):
            b, e = C.c_size_t(), C.c_size_t()
            lib.ketogpu_multi_range(n, parts, i, C.byref(b), C.byref(e))
            out.append((b.value, e.value))
        return out

    def check_ids(self, roots, targets, with_flags=False):
        roots = np.ascontiguousarray(roots, dtype=np.uint32)
        targets = np.ascontiguousarray(targets, dtype=np.uint32)
        n = len(roots)
        words = max((n + 63) // 64, 1)
        ab = np.zeros(words, dtype=np.uint64)
        fb = np.zeros(words, dtype=np.uint64)
        L.check(self.L.ketogpu_multi_check_ids(self.h, roots.ctypes.data, targets.ctypes.data, n, ab.ctypes.data,
                                               fb.ctypes.data))
        allowed = unpack_bits(ab, n)
        return (allowed, unpack_bits(fb, n)) if with_flags else allowed

    def check_ids_raw(self, roots_ptr, targets_ptr, n, allowed_ptr, flagged_ptr=None):
        """the C call on caller-owned (e.g. pinned) buffers, no conversions (benchmarks)"""
        L.check(self.L.ketogpu_multi_check_ids(self.h, roots_ptr, targets_ptr, n, allowed_ptr, flagged_ptr))

    def last_stats(self, i=0):
        return self.engine(i).last_stats()

    def engine(self, i):
        """the engine of device slot i (a borrowed view: statistics, HBM-resident queries)"""
        h = self.L.ketogpu_multi_engine(self.h, i)
        if not h:
            raise IndexError(i)
        return Engine.borrowed(h, self.snapshot, self)

    def close(self):
        if getattr(self, "h", None):
            self.L.ketogpu_multi_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


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

    def run(self, pipelined=False):
        """one batch call; pipelined: ketogpu_queries_run_async — returns True when the call
        was only enqueued (results complete after download() or Engine.wait())"""
        if not pipelined:
            L.check(self.e.L.ketogpu_queries_run(self.e.h, self.h))
            return False
        q = C.c_int(0)
        L.check(self.e.L.ketogpu_queries_run_async(self.e.h, self.h, C.byref(q)))
        return bool(q.value)

    def download(self, with_flags=False):
        words = max((self.n + 63) // 64, 1)
        ab = np.zeros(words, dtype=np.uint64)
        fb = np.zeros(words, dtype=np.uint64)
        L.check(self.e.L.ketogpu_queries_download(self.e.h, self.h, ab.ctypes.data, fb.ctypes.data))
        return (unpack_bits(ab, self.n), unpack_bits(fb, self.n)) if with_flags else unpack_bits(ab, self.n)

    def download_words(self):
        """the raw result and flag words (ceil(n/64) each)"""
        words = max((self.n + 63) // 64, 1)
        ab = np.zeros(words, dtype=np.uint64)
        fb = np.zeros(words, dtype=np.uint64)
        L.check(self.e.L.ketogpu_queries_download(self.e.h, self.h, ab.ctypes.data, fb.ctypes.data))
        return ab, fb

    def close(self):
        if getattr(self, "h", None):
            self.e.L.ketogpu_queries_free(self.h)
            self.h = None

    def __del__(self):
        self.close()
