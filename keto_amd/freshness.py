"""Read-your-writes over immutable snapshots (R14).

The reference reads the database on every check, so a check issued after a successful
write sees it (internal/persistence/sql/relationtuples.go:271-278 then :203-258).  The
GPU engines answer from an immutable device snapshot instead, so writes go through a
VersionedEngine: `transact` applies the batch to the current snapshot
(ketogpu_snapshot_apply: same ORDER BY, commit_time and delete-all-duplicates rules as
the SQL write path), builds the engines of the new version and swaps them in before it
returns the new version number.  Every check or expand issued after `transact` returned
runs on a version that contains the write; a check in flight keeps the version it
started on (the old engine lives until its last reference is dropped).  Unknown
namespace names fail the whole transaction (GetNamespaceByName -> ErrNotFound), as in
the reference.

Cost.  On a writable snapshot (Snapshot(..., writable=True): device rows with free slots,
KETOGPU_BUILD_WRITABLE) a transaction is written IN PLACE (ketogpu_snapshot_write): the
touched groups' host rows and the touched device rows are rewritten and the engine uploads
just those rows (ketogpu_engine_sync) before `transact` returns — O(rows of the touched
groups), not O(graph).  A batch the free slots cannot hold (a new group, an expandable node
becoming interior, a full row, ...; include/ketogpu.h KETOGPU_WRITE_*) falls back to the
rebuild below, which lays the rows out with fresh free slots.  On other snapshots every
transaction rebuilds: O(rows) host work plus one device-graph upload.  `last_write`
reports which path the last transaction took and its cost.
"""
import threading
import time

from . import _lib as L
from . import check, expand, persistence
from .relationtuple import InternalRelationTuple, NilSubject


class _Failed:
    """stands in for the check engine after a committed write could reach no device copy"""

    def __init__(self, sync_err, rebuild_err):
        self.why = f"sync failed ({sync_err}); rebuild failed ({rebuild_err})"

    def __getattr__(self, name):
        def fail(*a, **k):
            raise L.KetoError(L.EDEVICE, "no engine holds the last committed write: " + self.why)
        return fail


class VersionedEngine:
    def __init__(self, snapshot, device=0, **engine_opts):
        self.device = device
        self.engine_opts = engine_opts
        self._lock = threading.Lock()  # one writer at a time
        self.version = 0
        self.last_write = None
        self._install(snapshot)

    def _install(self, snapshot):
        eng = check.Engine(snapshot, device=self.device, **self.engine_opts)
        state = (snapshot, eng, expand.Engine(snapshot))
        self._state = state  # one reference swap: readers see the old or the new version
        return state

    # ---------------------------------------------------------------- writes
    def _rows(self, tuples):
        rows = []
        for t in tuples:
            if isinstance(t, dict):
                t = InternalRelationTuple.from_dict(t)
            if t.subject is None:
                raise NilSubject("subject is not allowed to be nil")
            rows.extend(persistence.rows_from_tuples(self._state[0].namespaces, [t]))
        return rows

    def transact(self, insert=(), delete=()):
        """TransactRelationTuples: insert, then delete; returns the new version"""
        with self._lock:
            snap, eng = self._state[0], self._state[1]
            ins, dele = self._rows(insert), self._rows(delete)
            t0 = time.perf_counter()
            res = snap.write(ins, dele)  # reason "not_writable" on a snapshot without free slots
            if res["applied"]:
                # the write is in the shared host snapshot from here on: it is committed
                # whatever happens to the device copy, so a failed sync must not turn into
                # a failed transaction (TransactRelationTuples is all-or-nothing)
                try:
                    sync_ms, rows = eng.sync()  # the patched device rows, before returning
                except L.KetoError as err:
                    failed = self._recover(snap, err)
                    self.last_write = dict(res, path="in_place+rebuild" if failed is None else "in_place+failed",
                                           sync_error=str(err), ms=(time.perf_counter() - t0) * 1e3)
                    if failed is not None:
                        self.last_write["engine_error"] = failed
                else:
                    self.last_write = dict(res, path="in_place", sync_ms=sync_ms, synced_rows=rows,
                                           ms=(time.perf_counter() - t0) * 1e3)
            else:
                self._install(snap.apply(ins, dele))
                self.last_write = {"applied": False, "reason": res["reason"], "path": "rebuild",
                                   "ms": (time.perf_counter() - t0) * 1e3}
            self.version += 1
            return self.version

    def _recover(self, snap, err):
        """the device sync of a committed in-place write failed: serve the written snapshot
        from a freshly built engine (a full upload of its rows).  If that fails too, the
        engine is left FAILED: every later read raises instead of answering from a device
        copy that lacks the committed write.  The transaction itself stands either way (it
        is in the shared snapshot), so transact returns its version; returns None, or the
        FAILED engine's error message"""
        try:
            self._install(snap.apply((), ()))
            return None
        except L.KetoError as err2:
            self._state = (snap, _Failed(err, err2), expand.Engine(snap))
            return (f"write committed, but no engine holds it: sync failed ({err}), rebuild failed ({err2}); "
                    f"checks raise until the next write")

    def reload_namespaces(self, namespaces):
        """Keto's KeyNamespaces reload (internal/driver/config/provider.go:87-110): the next
        version holds the same rows under the new configuration (page poisoning and name
        resolution follow it); engines swap before this returns the new version"""
        with self._lock:
            self._install(self._state[0].set_namespaces(namespaces))
            self.version += 1
            return self.version

    def WriteRelationTuples(self, *tuples):
        return self.transact(insert=tuples)

    def DeleteRelationTuples(self, *tuples):
        return self.transact(delete=tuples)

    # ----------------------------------------------------------------- reads
    @property
    def snapshot(self):
        return self._state[0]

    def SubjectIsAllowed(self, t):
        return self._state[1].SubjectIsAllowed(t)

    def check_many(self, tuples):
        return self._state[1].check_many(tuples)

    def BuildTree(self, subject, rest_depth):
        return self._state[2].BuildTree(subject, rest_depth)
