"""Partitioned mode: batched checks over a hash-partitioned graph, one process per GPU.

BASELINE.json config #5 / SURVEY.md 8(e): a graph that fits neither one GPU nor one host.

Loading (Shard.load; libketogpu's ketogpu_shard_*): every rank streams the ONE ordered
row read of the network (internal/persistence/sql/relationtuples.go:203-258) and keeps
what it owns — the rows of the groups it owns and the rows whose subject it owns — then
the ranks exchange node ids once (all_gather of the per-class counts, all_to_all of node
hashes and their ids) and check for shared Subject.String() keys (R4).  No rank interns
or holds the whole graph: host memory per rank is O(rows / world).

Checking (PartitionedEngine): a round of up to 64*W requests is a multi-source BFS whose
levels exchange (word, node, mask) records between ranks:

    begin -> { emit -> all_to_all -> apply -> all_reduce(frontier) ; stop at 0 -> expand }
          -> pull_emit -> all_to_all -> pull_answer -> end -> all_reduce(MAX) of the hit bits

(three collectives per level: the counts of the all_to_all, its records, the frontier
all-reduce; the steps' statuses ride in the counts and the all-reduce)

The device steps are libketogpu's ketogpu_part_* (keto_amd/csrc/partition.hip); this
module is the exchange: torch.distributed collectives on device tensors (backend "nccl" =
RCCL over xGMI), or through host memory for gloo.  It answers exactly what
check.Engine.check_ids answers for the same network (the same reachability formula, R2:
no depth cutoff).  A step that fails on one rank fails the round on every rank: each
step's status travels in the next collective every rank makes anyway, so no rank is left
waiting in a collective its peers will never enter.
"""
import ctypes as C
import time

import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L

REC_COLS = 4  # a 16-byte ketogpu_record as 4 int32 columns
FORWARD, BACKWARD = 0, 1  # include/ketogpu.h KETOGPU_PART_FORWARD / _BACKWARD
NOT_OWNED = 1 << 32       # ketogpu_shard_resolve_batch's KETOGPU_NODE_NOT_OWNED, widened for MIN


def records_to_tensor(a, b, m):
    """numpy (a u32, b u32, m u64) -> int32 tensor (n, 4) in ketogpu_record layout"""
    rec = np.empty(len(a), dtype=[("a", "<u4"), ("b", "<u4"), ("m", "<u8")])
    rec["a"], rec["b"], rec["m"] = a, b, m
    return torch.from_numpy(rec.view(np.int32).reshape(-1, REC_COLS).copy())


def tensor_to_records(t):
    """int32 tensor (n, 4) -> (a, b, m) numpy arrays"""
    rec = np.ascontiguousarray(t.cpu().numpy()).view([("a", "<u4"), ("b", "<u4"), ("m", "<u8")]).reshape(-1)
    return rec["a"].copy(), rec["b"].copy(), rec["m"].copy()


class Comm:
    """the collectives of one process group (or none: a single rank)"""

    def __init__(self, group=None):
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
            self.cuda = dist.get_backend(group) == "nccl"
        else:
            self.rank, self.world, self.cuda = 0, 1, False

    def device(self):
        return torch.device("cuda", torch.cuda.current_device()) if self.cuda else torch.device("cpu")

    def allreduce(self, vals, op="sum"):
        if self.world == 1:
            return [int(v) for v in vals]
        t = torch.tensor([int(v) for v in vals], dtype=torch.int64, device=self.device())
        dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op],
                        group=self.group)
        return [int(v) for v in t.tolist()]

    def allreduce_array(self, a, op):
        """numpy array (int64 or uint8), reduced elementwise"""
        if self.world == 1:
            return a
        t = torch.from_numpy(np.ascontiguousarray(a)).to(self.device())
        dist.all_reduce(t, op={"max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op], group=self.group)
        return t.cpu().numpy()

    def allgather(self, vals):
        """each rank's int list -> [rank][...]"""
        if self.world == 1:
            return [list(vals)]
        t = torch.tensor([int(v) for v in vals], dtype=torch.int64, device=self.device())
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [[int(v) for v in o.tolist()] for o in out]

    def alltoall(self, send, counts, cols=1):
        """send: numpy int64/uint64 array grouped by destination (counts per rank, in rows of
        `cols` values) -> (received array, counts received per source)"""
        if self.world == 1:
            return send, list(counts)
        dev = self.device()
        cnt = torch.tensor([int(c) for c in counts], dtype=torch.int64, device=dev)
        rcnt = torch.empty_like(cnt)
        dist.all_to_all_single(rcnt, cnt, group=self.group)
        rc = [int(x) for x in rcnt.tolist()]
        src = torch.from_numpy(np.ascontiguousarray(send).view(np.int64).reshape(-1, cols)).to(dev)
        recv = torch.empty((sum(rc), cols), dtype=torch.int64, device=dev)
        dist.all_to_all_single(recv, src, rc, [int(c) for c in counts], group=self.group)
        return recv.cpu().numpy().reshape(-1).view(send.dtype), rc

    def agree(self, code):
        """every rank's step status -> the largest (0 when all succeeded)"""
        return self.allreduce([code], "max")[0]


def _status(fn, *a):
    """run one local step: (0, result) or (KETOGPU_E* code, message)"""
    try:
        return 0, fn(*a)
    except L.KetoError as e:
        return e.code, str(e)


class Shard:
    """One rank's part of a partitioned network (ketogpu_shard_*), loaded collectively."""

    def __init__(self, handle, comm, namespaces):
        self.L = L.lib()
        self.h = handle
        self.comm = comm
        self.namespaces = namespaces

    @classmethod
    def load(cls, namespaces, batches, group=None, page_size=100, order="sqlite", salt=0x4B45544F, tries=3):
        """namespaces [(name, id)]; batches: a callable returning an iterator of row column
        dicts in the backend's ORDER BY order (the same stream on every rank).  Every rank
        calls this together."""
        comm = Comm(group)
        for attempt in range(tries):
            try:
                return cls._load_once(namespaces, batches, comm, page_size, order, salt + attempt)
            except L.KetoError as e:
                if e.code != L.ECOLLISION or attempt + 1 == tries:
                    raise
        raise AssertionError("unreachable")

    @classmethod
    def _load_once(cls, namespaces, batches, comm, page_size, order, salt):
        lib = L.lib()
        ns = [(n, int(i)) for n, i in namespaces]
        arr = (L.Namespace * max(len(ns), 1))(*[L.Namespace(i, L.b(n)) for n, i in ns])
        opts = L.ShardOpts(page_size, L.ORDERS[order], comm.rank, comm.world, salt)

        def stream():
            b = C.c_void_p()
            L.check(lib.ketogpu_shard_builder_new(arr, len(ns), C.byref(opts), C.byref(b)))
            try:
                for cols in batches():
                    L.check(lib.ketogpu_shard_builder_append(b, C.byref(L.row_batch(cols))))
            except BaseException:
                lib.ketogpu_shard_builder_free(b)
                raise
            h = C.c_void_p()
            L.check(lib.ketogpu_shard_builder_finish(b, C.byref(h)))
            return h

        code, h = _status(stream)
        err = comm.agree(code)
        if err:
            if not code and h:
                lib.ketogpu_shard_free(h)
            raise L.KetoError(err, h if code else "another rank failed to stream its shard")
        self = cls(h, comm, ns)
        try:
            self._exchange()
        except BaseException:
            self.close()
            raise
        return self

    def _step(self, fn, *a):
        code, res = _status(fn, *a)
        err = self.comm.agree(code)
        if err:
            raise L.KetoError(err, res if code else "shard loading failed on another rank")
        return res

    def _exchange(self):
        lib, comm, h = self.L, self.comm, self.h
        counts = np.zeros(3, dtype=np.uint64)
        L.check(lib.ketogpu_shard_counts(h, counts.ctypes.data))
        allc = np.array(comm.allgather(counts.tolist()), dtype=np.uint64).reshape(-1)
        self._step(lambda: L.check(lib.ketogpu_shard_set_layout(h, allc.ctypes.data)))
        # node ids: hashes to their owners, ids back in the same order
        nq = int(lib.ketogpu_shard_query_count(h))
        q = np.zeros(max(nq, 1), dtype=np.uint64)
        qc = np.zeros(comm.world, dtype=np.uint64)
        L.check(lib.ketogpu_shard_queries(h, q.ctypes.data, nq, qc.ctypes.data))
        recv, rc = comm.alltoall(q[:nq], qc.tolist())
        ans = np.zeros(max(len(recv), 1), dtype=np.uint64)  # u32 ids carried in u64 lanes
        ids32 = np.zeros(max(len(recv), 1), dtype=np.uint32)
        self._step(lambda: L.check(lib.ketogpu_shard_answer(h, np.ascontiguousarray(recv).ctypes.data, len(recv),
                                                             ids32.ctypes.data)))
        ans[:len(recv)] = ids32[:len(recv)]
        back, _ = comm.alltoall(ans[:len(recv)], rc)
        mine = np.ascontiguousarray(np.asarray(back, dtype=np.uint64).astype(np.uint32))
        self._step(lambda: L.check(lib.ketogpu_shard_apply(h, mine.ctypes.data if nq else None, nq)))
        # R4: shared Subject.String() keys
        nc = int(lib.ketogpu_shard_claim_count(h))
        pairs = np.zeros(max(2 * nc, 2), dtype=np.uint64)
        pc = np.zeros(comm.world, dtype=np.uint64)
        L.check(lib.ketogpu_shard_claims(h, pairs.ctypes.data, nc, pc.ctypes.data))
        got, _ = comm.alltoall(pairs[:2 * nc], pc.tolist(), cols=2)
        got = np.ascontiguousarray(got, dtype=np.uint64)
        amb = C.c_uint64()
        self._step(lambda: L.check(lib.ketogpu_shard_check_claims(h, got.ctypes.data, len(got) // 2, C.byref(amb))))
        total = comm.allreduce([amb.value])[0]
        if total:
            raise L.KetoError(L.EINVAL, f"partitioned loader: {total} Subject.String() keys are shared by two nodes "
                                        "(R4); load this network with the whole-graph snapshot")

    def stats(self):
        st = L.ShardStats()
        L.check(self.L.ketogpu_shard_stats_get(self.h, C.byref(st)))
        return st.as_dict()

    def view(self):
        """numpy copies of the rank's device rows (ketogpu_shard_view)"""
        v = L.ShardGraph()
        L.check(self.L.ketogpu_shard_view(self.h, C.byref(v)))

        def arr(p, n, dt):
            return np.ctypeslib.as_array(p, (n,)).copy() if n else np.zeros(0, dtype=dt)
        out = {k: getattr(v, k) for k in ("rank", "world", "num_interior", "num_expandable", "num_nodes",
                                          "owned_interior", "owned_expandable", "owned_nodes")}
        for name, rows in (("lf", v.owned_expandable), ("lr", v.owned_nodes), ("lb", v.owned_interior)):
            off = arr(getattr(v, name + "_off"), rows + 1, np.uint64)
            out[name + "_off"] = off
            out[name + "_col"] = arr(getattr(v, name + "_col"), int(off[-1]), np.uint32)
        return out

    def resolve_batch(self, cols):
        """request columns (persistence.request_columns, or a ready L.RequestBatch) ->
        (roots, targets, status): every rank resolves the nodes it owns, the owners'
        answers are combined (all_reduce MIN)"""
        rb = cols if isinstance(cols, L.RequestBatch) else L.request_batch(cols)
        n = rb.n
        r = np.zeros(max(n, 1), dtype=np.uint32)
        t = np.zeros(max(n, 1), dtype=np.uint32)
        st = np.zeros(max(n, 1), dtype=np.int32)
        code, msg = _status(lambda: L.check(self.L.ketogpu_shard_resolve_batch(self.h, C.byref(rb), r.ctypes.data,
                                                                                t.ctypes.data, st.ctypes.data)))
        err = self.comm.agree(code)
        if err:
            raise L.KetoError(err, msg if code else "request resolution failed on another rank")
        both = np.concatenate([r[:n], t[:n]]).astype(np.int64)
        both[both == L.NODE_NOT_OWNED] = NOT_OWNED
        both = self.comm.allreduce_array(both, "min")
        both[both == NOT_OWNED] = L.NODE_NONE  # (no owner: cannot happen; treated as absent)
        return both[:n].astype(np.uint32), both[n:].astype(np.uint32), st[:n].copy()

    def close(self):
        if getattr(self, "h", None):
            self.L.ketogpu_shard_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


class DevicePartition:
    """One rank's device steps (ketogpu_part_*); records travel in int32 tensors on its GPU."""

    def __init__(self, shard, device=0, record_capacity=1 << 22, max_words_per_round=0, state_budget_bytes=0):
        self.L = L.lib()
        self.shard = shard  # keeps the host shard alive
        self.world = shard.comm.world
        self.device = torch.device("cuda", device)
        opts = L.PartOpts(device, shard.comm.rank, shard.comm.world, record_capacity, max_words_per_round,
                          state_budget_bytes)
        h = C.c_void_p()
        L.check(self.L.ketogpu_part_new(shard.h, C.byref(opts), C.byref(h)))
        self.h = h
        self.cap = record_capacity
        self.send = torch.empty((self.cap, REC_COLS), dtype=torch.int32, device=self.device)
        self.counts = np.zeros(max(self.world, 1), dtype=np.uint64)
        self._req = None

    def owner(self, v):
        return int(self.L.ketogpu_part_owner(self.h, int(v)))

    def round_words(self):
        return int(self.L.ketogpu_part_round_words(self.h))

    def begin(self, roots, targets, direction=FORWARD):
        self._req = (np.ascontiguousarray(roots, dtype=np.uint32), np.ascontiguousarray(targets, dtype=np.uint32))
        r, t = self._req
        return self._rc(self.L.ketogpu_part_begin_dir(self.h, r.ctypes.data, t.ctypes.data, len(r), direction))

    def _rc(self, rc):
        """a step's status: 0, or its KETOGPU_E* code (ENOMEM = retry with a smaller round)"""
        if rc and rc != L.ENOMEM:
            self.error = (rc, (self.L.ketogpu_last_error() or b"").decode("utf-8", "replace"))
        return rc

    def _pack(self, fn):
        rc = self._rc(fn(self.h, self.send.data_ptr(), self.cap, self.counts.ctypes.data))
        if rc:
            return rc, self.send[:0], [0] * self.world
        counts = [int(x) for x in self.counts[:self.world]]
        return 0, self.send[:sum(counts)], counts

    def emit(self):
        return self._pack(self.L.ketogpu_part_emit)

    def pull_emit(self):
        return self._pack(self.L.ketogpu_part_pull_emit)

    def _recv(self, recv):
        recv = recv.to(self.device).contiguous()
        torch.cuda.current_stream(self.device).synchronize()  # the exchange wrote it on torch's stream
        return recv

    def apply(self, recv):
        recv = self._recv(recv)
        fr = C.c_uint64()
        rc = self._rc(self.L.ketogpu_part_apply(self.h, recv.data_ptr() if len(recv) else None, len(recv),
                                                C.byref(fr)))
        return rc, (fr.value if not rc else 0)

    def expand(self):
        return self._rc(self.L.ketogpu_part_expand(self.h))

    def pull_answer(self, recv):
        recv = self._recv(recv)
        return self._rc(self.L.ketogpu_part_pull_answer(self.h, recv.data_ptr() if len(recv) else None, len(recv)))

    def end(self, n):
        bits = np.zeros(max((n + 63) // 64, 1), dtype=np.uint64)
        L.check(self.L.ketogpu_part_end(self.h, bits.ctypes.data))
        return bits

    def abort(self):
        L.check(self.L.ketogpu_part_abort(self.h))

    def stats(self):
        st = L.PartStats()
        L.check(self.L.ketogpu_part_stats_get(self.h, C.byref(st)))
        return st.as_dict()

    def set_timing(self, on):
        """bracket every kernel launch with hipEvents (a measurement pass)"""
        L.check(self.L.ketogpu_part_set_timing(self.h, 1 if on else 0))

    def close(self):
        if getattr(self, "h", None):
            self.L.ketogpu_part_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


class PartitionedEngine:
    """check_ids over the partitioned graph.  Every rank calls check_ids with the same
    (roots, targets) and gets the full answer.  `local` is the rank's step implementation
    (DevicePartition over `shard` by default)."""

    def __init__(self, shard, device=0, local=None, direction="auto", **opts):
        """direction: "forward" (grow the roots' closures), "backward" (grow the targets'
        ancestor sets) or "auto": the first two full rounds run one direction each, timed
        (max over ranks, so every rank decides alike), and the faster is kept"""
        if direction not in ("auto", "forward", "backward"):
            raise ValueError("direction must be auto, forward or backward")
        self.direction = {"forward": FORWARD, "backward": BACKWARD}.get(direction)
        self._trial = {}  # direction -> ns per request of its trial round
        self._per = {FORWARD: 1 << 62, BACKWARD: 1 << 62}  # requests per round after overflow retries
        self.shard = shard
        self.comm = shard.comm if shard is not None else Comm()
        self.rank, self.world, self.comm_cuda = self.comm.rank, self.comm.world, self.comm.cuda
        self.local = local if local is not None else DevicePartition(shard, device, **opts)
        self.levels = 0
        self.retries = 0
        self.records = 0

    def _exchange(self, st, send, counts):
        """records to their owners.  The step's status travels with the counts: a rank whose
        step failed sends -code as every count, so every rank learns it from the one counts
        exchange it makes anyway.  -> (status agreed by all ranks, received records)"""
        if self.world == 1:
            self.records += int(sum(counts)) if not st else 0
            return st, send
        cdev = self.comm.device()
        cnt = torch.tensor([-st] * self.world if st else counts, dtype=torch.int64, device=cdev)
        rcnt = torch.empty_like(cnt)
        dist.all_to_all_single(rcnt, cnt, group=self.comm.group)
        rc = [int(x) for x in rcnt.tolist()]
        bad = max([-c for c in rc if c < 0] + [st])
        if bad:
            return bad, None
        self.records += int(sum(counts))
        recv = torch.empty((sum(rc), REC_COLS), dtype=torch.int32, device=cdev)
        dist.all_to_all_single(recv, send.to(cdev), rc, list(counts), group=self.comm.group)
        return 0, recv

    def _frontier(self, frontier, st):
        """one all-reduce per level: the frontier total and every rank's step status (per-code
        counts, so the largest failing code is known everywhere)"""
        v = [frontier] + [1 if st == c else 0 for c in range(1, 6)]
        if self.world > 1:
            v = self.comm.allreduce(v, "sum")
        codes = [c for c in range(1, 6) if v[c]]
        return v[0], (max(codes) if codes else 0)

    def _fail(self, code):
        """a step failed on some rank: every rank aborts the round; ENOMEM means retry with
        fewer requests (None), anything else is raised on every rank"""
        self.local.abort()
        if code == L.ENOMEM:
            return None
        err = getattr(self.local, "error", None)
        raise L.KetoError(code, err[1] if err and err[0] == code else "a partition step failed on another rank")

    # -------------------------------------------------------------------- rounds
    def _round(self, roots, targets, direction):
        """one round; None when a rank's buffers overflowed (every rank aborts).  Per level
        three collectives: counts (carrying the step status), records, and the frontier
        all-reduce (carrying the apply status)"""
        loc = self.local
        pending = loc.begin(roots, targets, direction) or 0  # reported with the first emit
        while True:
            st, send, counts = loc.emit()
            code, recv = self._exchange(pending or st, send, counts)
            if code:
                return self._fail(code)
            st, frontier = loc.apply(recv)
            total, code = self._frontier(frontier, st)
            if code:
                return self._fail(code)
            self.levels += 1
            if total == 0:  # no rank has a frontier left: the closure is complete
                break
            pending = loc.expand() or 0  # reported with the next emit
        st, send, counts = loc.pull_emit()
        code, recv = self._exchange(st, send, counts)
        if code:
            return self._fail(code)
        st = loc.pull_answer(recv) or 0
        bits = loc.end(len(roots)) if not st else None
        # one byte (0/1) per request: an int64 per request cost ~3 ms of host time per 10^6
        # requests (unpack, widen, narrow) and 8x the bytes of the all-reduce below
        hit = np.zeros(len(roots), dtype=np.uint8) if st else \
            np.unpackbits(bits.view(np.uint8), bitorder="little")[:len(roots)]
        if self.world > 1:  # the answer is the OR (MAX) of the ranks' hits; the last lane
            # carries the ranks' pull_answer status (MAX: the largest failing code, < 256)
            hit = self.comm.allreduce_array(np.concatenate([hit, np.array([st], dtype=np.uint8)]), "max")
            code = int(hit[-1])
            hit = hit[:-1]
            if code:
                return self._fail(code)
        elif st:
            return self._fail(st)
        return hit.view(bool)

    def check_ids(self, roots, targets):
        roots = np.ascontiguousarray(roots, dtype=np.uint32)
        targets = np.ascontiguousarray(targets, dtype=np.uint32)
        n = len(roots)
        top = self.comm.allreduce([self.local.round_words() * 64], "min")[0]
        out = np.zeros(n, dtype=bool)
        i = 0
        while i < n:
            if self.direction is None:
                # auto: both directions run the SAME first round (equal work), timed (max over
                # ranks, so every rank decides alike); the faster direction is kept
                m = min(top, self._per[FORWARD], self._per[BACKWARD], n - i)
                got = {}
                for d in (FORWARD, BACKWARD):
                    t0 = time.perf_counter()
                    got[d] = self._round(roots[i:i + m], targets[i:i + m], d)
                    ns = int((time.perf_counter() - t0) * 1e9 / max(m, 1))
                    self._trial[d] = self.comm.allreduce([ns], "max")[0]
                if got[FORWARD] is None or got[BACKWARD] is None:
                    self._trial = {}
                    for d in (FORWARD, BACKWARD):
                        self._shrink(d, m)
                    continue
                if not np.array_equal(got[FORWARD], got[BACKWARD]):
                    raise L.KetoError(L.EDEVICE, "partition: forward and backward rounds disagree")
                self.direction = min(self._trial, key=lambda k: (self._trial[k], k))
                out[i:i + m] = got[FORWARD]
                i += m
                continue
            d = self.direction
            m = min(top, self._per[d], n - i)  # a round size that overflowed stays halved for later calls
            got = self._round(roots[i:i + m], targets[i:i + m], d)
            if got is None:
                self._shrink(d, m)
                continue
            out[i:i + m] = got
            i += m
        return out

    def check_requests(self, cols):
        """SubjectIsAllowed for request columns (persistence.request_columns): resolution by
        the owners, then check_ids; nil subjects raise like the single-GPU engine"""
        roots, targets, status = self.shard.resolve_batch(cols)
        if (status == L.EINVAL).any():
            from .relationtuple import NilSubject
            raise NilSubject("subject is not allowed to be nil")
        # a wildcard root (R5: empty namespace/object/relation, relationtuples.go:218-236)
        # matches every group it filters to; the shard has no node for that union, and the
        # reference may answer True there, so it is refused rather than answered False
        bad = np.flatnonzero(self.comm.allreduce_array(status.astype(np.int64), "max") == L.ENOTFOUND)
        if len(bad):
            raise L.KetoError(L.EINVAL, f"partitioned engine: {len(bad)} requests have wildcard roots (first index "
                                        f"{int(bad[0])}); evaluate them with the whole-graph engine")
        return self.check_ids(roots, targets)

    def _shrink(self, d, m):
        if m <= 64:
            raise L.KetoError(L.ENOMEM, "partition buffers overflow for a single 64-request word")
        self._per[d] = max(64, (m // 2) // 64 * 64)
        self.retries += 1

    def close(self):
        close = getattr(self.local, "close", None)
        if close:
            close()
