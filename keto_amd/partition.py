"""Partitioned mode: batched checks over a hash-partitioned graph, one process per GPU.

BASELINE.json config #5 / SURVEY.md 8(e): a graph that fits neither one GPU nor one host.

Loading (Shard.load; libketogpu's ketogpu_shard_*): every rank streams the ONE ordered
row read of the network (internal/persistence/sql/relationtuples.go:203-258) and keeps
what it owns — the rows of the groups it owns and the rows whose subject it owns — then
the ranks exchange node ids once and check for shared Subject.String() keys (R4), all in
one native call (ketogpu_shard_exchange).  No rank interns or holds the whole graph: host
memory per rank is O(rows / world).

Checking (PartitionedEngine): ONE native call per batch, ketogpu_part_check_ids
(keto_amd/csrc/part_round.cpp).  A round of up to 64*W requests is a multi-source BFS
whose levels exchange (word, node, mask) records between ranks:

    begin -> { emit -> [all-gather counts+status] -> [all-to-all records] -> apply -> expand }
          -> pull_emit -> [all-gather] -> [all-to-all] -> pull_answer -> end -> [all-gather bits]

two collectives per level, inside libketogpu: RCCL over xGMI between GPUs (grouped
ncclSend/ncclRecv, ncclAllGather on the partition's stream), or a host transport (this
module's gloo callbacks: the CPU tests, two ranks sharing one GPU).  It answers exactly
what check.Engine.check_ids answers for the same network (the same reachability formula,
R2: no depth cutoff).  A step that fails on one rank fails the round on every rank: its
status travels in the counts all-gather every rank makes anyway.

This module only sets the communicator up (NativeComm: the RCCL id broadcast once over the
torch.distributed group) and mirrors the reference's names; a Go host makes the same C
calls.
"""
import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L

FORWARD, BACKWARD = 0, 1  # include/ketogpu.h KETOGPU_PART_FORWARD / _BACKWARD


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
    def load(cls, namespaces, batches, group=None, page_size=100, order="sqlite", salt=0x4B45544F, tries=3,
             native_comm=None):
        """namespaces [(name, id)]; batches: a callable returning an iterator of row column
        dicts in the backend's ORDER BY order (the same stream on every rank).  Every rank
        calls this together.  native_comm: the NativeComm the id exchange (and later the
        engine) uses; default: RCCL on a nccl group, the host transport otherwise."""
        comm = Comm(group)
        for attempt in range(tries):
            try:
                return cls._load_once(namespaces, batches, comm, page_size, order, salt + attempt, native_comm)
            except L.KetoError as e:
                if e.code != L.ECOLLISION or attempt + 1 == tries:
                    raise
        raise AssertionError("unreachable")

    @classmethod
    def _load_once(cls, namespaces, batches, comm, page_size, order, salt, native_comm=None):
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
        if native_comm is not None:
            self._ncomm = {"auto": native_comm}
        try:
            self._exchange()
        except BaseException:
            self.close()
            raise
        return self

    def _exchange(self):
        """node ids and R4 claims between the ranks: ketogpu_shard_exchange over the
        shard's communicator (every step's status agreed by all ranks)"""
        L.check(self.L.ketogpu_shard_exchange(self.h, self.native_comm().handle))

    def native_comm(self, device=None, host_steps=False):
        """the ketogpu_comm of this shard's ranks (made once; RCCL on a nccl group, where
        `device` is this rank's GPU — host steps, tests only, use the host transport)"""
        key = "transport" if host_steps and self.comm.world > 1 else "auto"
        if getattr(self, "_ncomm", None) is None:
            self._ncomm = {}
        if key not in self._ncomm:
            if self.comm.cuda and key == "auto" and self.comm.world > 1:
                self._ncomm[key] = NativeComm(self.comm.group, device, kind="rccl")
            else:
                self._ncomm[key] = NativeComm(self.comm.group, device, kind=None if self.comm.world == 1 else "transport")
        return self._ncomm[key]

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

    def resolve_batch(self, cols, comm=None):
        """request columns (persistence.request_columns, or a ready L.RequestBatch) ->
        (roots, targets, status): every rank resolves the nodes it owns, the owners'
        answers win (ketogpu_part_resolve_batch)"""
        rb = cols if isinstance(cols, L.RequestBatch) else L.request_batch(cols)
        n = rb.n
        r = np.zeros(max(n, 1), dtype=np.uint32)
        t = np.zeros(max(n, 1), dtype=np.uint32)
        st = np.zeros(max(n, 1), dtype=np.int32)
        comm = comm or self.native_comm()
        L.check(self.L.ketogpu_part_resolve_batch(self.h, comm.handle, C.byref(rb), r.ctypes.data, t.ctypes.data,
                                                  st.ctypes.data))
        return r[:n].copy(), t[:n].copy(), st[:n].copy()

    def close(self):
        if getattr(self, "h", None):
            self.L.ketogpu_shard_free(self.h)
            self.h = None
        self._ncomm = {}  # communicators close when their last user drops them

    def __del__(self):
        self.close()


class NativeComm:
    """a ketogpu_comm for the ranks of a torch.distributed group (include/ketogpu.h "whole
    rounds"): RCCL inside libketogpu when the group's backend is nccl (the id travels once
    over the group), else a host transport over the group (gloo) whose callbacks run the
    group's collectives.  world 1 without `kind`: no communicator at all (handle None)."""

    def __init__(self, group=None, device=None, kind="auto"):
        self.L = L.lib()
        self.py = Comm(group)
        self.rank, self.world = self.py.rank, self.py.world
        self.h = None
        self._keep = None
        if kind == "auto":
            kind = None if self.world == 1 else ("rccl" if self.py.cuda else "transport")
        if kind == "rccl":
            dev = torch.cuda.current_device() if device is None else int(device)
            uid = (C.c_uint8 * L.COMM_ID_BYTES)()
            if self.rank == 0:
                L.check(self.L.ketogpu_comm_unique_id(uid))
            if self.world > 1:
                t = torch.tensor(list(bytes(uid)), dtype=torch.uint8, device=self.py.device())
                dist.broadcast(t, dist.get_global_rank(group, 0) if group is not None else 0, group=group)
                uid = (C.c_uint8 * L.COMM_ID_BYTES)(*t.cpu().tolist())
            h = C.c_void_p()
            L.check(self.L.ketogpu_comm_new(uid, self.rank, self.world, dev, C.byref(h)))
            self.h = h
        elif kind == "transport":
            self._keep = _GroupTransport(self.py)
            h = C.c_void_p()
            L.check(self.L.ketogpu_comm_from_transport(C.byref(self._keep.vt), C.byref(h)))
            self.h = h
        elif kind is not None:
            raise ValueError("kind: auto, rccl or transport")
        self.kind = kind

    @property
    def handle(self):
        return self.h

    def stats(self):
        """RCCL calls this communicator made (ketogpu_comm_stats_get)"""
        st = L.CommStats()
        if self.h:
            L.check(self.L.ketogpu_comm_stats_get(self.h, C.byref(st)))
        return st.as_dict()

    def close(self):
        if getattr(self, "h", None):
            self.L.ketogpu_comm_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


class _GroupTransport:
    """ketogpu_transport callbacks over a torch.distributed group (host memory).  A callback
    that raises returns 1: the library then fails the call on this rank (its peers fail in
    the same collective)."""

    def __init__(self, comm):
        self.c = comm
        self.error = None

        def guard(fn):
            def run(*a):
                try:
                    fn(*a)
                    return 0
                except Exception as e:  # noqa: BLE001 - reported through the status code
                    self.error = e
                    return 1
            return run

        def allgather(_ctx, send, recv, nbytes):
            dev = self.c.device()
            t = torch.frombuffer(bytearray(C.string_at(send, nbytes)) if nbytes else bytearray(1),
                                 dtype=torch.uint8)[:nbytes].to(dev)
            out = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(self.c.world)]
            dist.all_gather(out, t, group=self.c.group)
            data = b"".join(bytes(o.cpu().numpy()) for o in out)
            C.memmove(recv, data, len(data))

        def alltoallv(_ctx, send, sb, recv, rb):
            w = self.c.world
            sbytes = [int(sb[i]) for i in range(w)]
            rbytes = [int(rb[i]) for i in range(w)]
            dev = self.c.device()
            src = torch.frombuffer(bytearray(C.string_at(send, sum(sbytes))) if sum(sbytes) else bytearray(1),
                                   dtype=torch.uint8)[:sum(sbytes)].to(dev)
            dst = torch.empty(sum(rbytes), dtype=torch.uint8, device=dev)
            dist.all_to_all_single(dst, src, rbytes, sbytes, group=self.c.group)
            if sum(rbytes):
                C.memmove(recv, bytes(dst.cpu().numpy()), sum(rbytes))

        def allreduce_u32(_ctx, buf, n, op):
            a = np.ctypeslib.as_array(buf, (n,)) if n else np.zeros(0, np.uint32)
            t = torch.from_numpy(a.astype(np.int64)).to(self.c.device())
            dist.all_reduce(t, op=dist.ReduceOp.MIN if op == L.REDUCE_MIN else dist.ReduceOp.MAX, group=self.c.group)
            if n:
                a[:] = t.cpu().numpy().astype(np.uint32)

        self.fns = (L.ALLGATHER_FN(guard(allgather)), L.ALLTOALLV_FN(guard(alltoallv)),
                    L.ALLREDUCE_FN(guard(allreduce_u32)))
        self.vt = L.Transport(None, comm.rank, comm.world, *self.fns)


class DevicePartition:
    """One rank's HIP partition (ketogpu_part_*): the device rows of its shard and the
    traversal state; its steps are driven by the native round (ketogpu_part_engine)."""

    def __init__(self, shard, device=0, record_capacity=1 << 22, max_words_per_round=0, state_budget_bytes=0):
        self.L = L.lib()
        self.shard = shard  # keeps the host shard alive
        self.world = shard.comm.world
        opts = L.PartOpts(device, shard.comm.rank, shard.comm.world, record_capacity, max_words_per_round,
                          state_budget_bytes)
        h = C.c_void_p()
        L.check(self.L.ketogpu_part_new(shard.h, C.byref(opts), C.byref(h)))
        self.h = h
        self.cap = record_capacity

    def owner(self, v):
        return int(self.L.ketogpu_part_owner(self.h, int(v)))

    def round_words(self):
        return int(self.L.ketogpu_part_round_words(self.h))

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


DIRECTIONS = {"auto": L.PART_AUTO, "forward": FORWARD, "backward": BACKWARD}


class PartitionedEngine:
    """check_ids over the partitioned graph: ONE native call per batch
    (ketogpu_part_check_ids: the level loop, the collectives and the overflow retries run
    inside libketogpu — RCCL between GPUs).  Every rank calls check_ids with the same
    (roots, targets) and gets the full answer.  `local` (tests only) is an object whose
    vtable() gives host steps (include/ketogpu.h ketogpu_part_steps) to drive instead of
    the HIP partition."""

    def __init__(self, shard, device=0, local=None, direction="auto", comm=None, **opts):
        """direction: "forward" (grow the roots' closures), "backward" (grow the targets'
        ancestor sets) or "auto": the first round runs once in each direction, timed (max
        over ranks, so every rank decides alike), and the faster is kept.  comm: a
        NativeComm (default: the shard's)."""
        if direction not in DIRECTIONS:
            raise ValueError("direction must be auto, forward or backward")
        self.L = L.lib()
        self.shard = shard
        self.comm = shard.comm if shard is not None else Comm()
        self.rank, self.world = self.comm.rank, self.comm.world
        if comm is None:
            comm = shard.native_comm(device, host_steps=local is not None)
        self.ncomm = comm
        eopts = L.PartEngineOpts(DIRECTIONS[direction], int(opts.get("record_capacity", 0)) if local is None else 0)
        h = C.c_void_p()
        if local is None:
            self.local = DevicePartition(shard, device, **opts)
            L.check(self.L.ketogpu_part_engine_new(self.local.h, comm.handle, C.byref(eopts), C.byref(h)))
        else:
            self.local = local
            self._vt = local.vtable()
            L.check(self.L.ketogpu_part_engine_new_steps(C.byref(self._vt), comm.handle, C.byref(eopts), C.byref(h)))
        self.h = h

    def stats(self):
        st = L.PartEngineStats()
        L.check(self.L.ketogpu_part_engine_stats_get(self.h, C.byref(st)))
        return st.as_dict()

    @property
    def direction(self):
        d = self.stats()["direction"]
        return None if d == L.PART_AUTO else d

    @property
    def _trial(self):
        t = self.stats()["trial_ns"]
        return {FORWARD: t[0], BACKWARD: t[1]} if any(t) else {}

    @property
    def retries(self):
        return self.stats()["retries"]

    @property
    def records(self):
        return self.stats()["records_sent"]

    @property
    def levels(self):
        return self.stats()["levels"]

    def check_ids(self, roots, targets):
        roots = np.ascontiguousarray(roots, dtype=np.uint32)
        targets = np.ascontiguousarray(targets, dtype=np.uint32)
        n = len(roots)
        bits = np.zeros(max((n + 63) // 64, 1), dtype=np.uint64)
        L.check(self.L.ketogpu_part_check_ids(self.h, roots.ctypes.data, targets.ctypes.data, n, bits.ctypes.data))
        return np.unpackbits(bits.view(np.uint8), bitorder="little")[:n].astype(bool)

    def check_requests(self, cols):
        """SubjectIsAllowed for request columns (persistence.request_columns): resolution by
        the owners (ketogpu_part_resolve_batch), then check_ids; nil subjects raise like the
        single-GPU engine"""
        roots, targets, status = self.shard.resolve_batch(cols, self.ncomm)
        if (status == L.EINVAL).any():
            from .relationtuple import NilSubject
            raise NilSubject("subject is not allowed to be nil")
        # a wildcard root (R5: empty namespace/object/relation, relationtuples.go:218-236)
        # matches every group it filters to; the shard has no node for that union, and the
        # reference may answer True there, so it is refused rather than answered False
        bad = np.flatnonzero(status == L.ENOTFOUND)
        if len(bad):
            raise L.KetoError(L.EINVAL, f"partitioned engine: {len(bad)} requests have wildcard roots (first index "
                                        f"{int(bad[0])}); evaluate them with the whole-graph engine")
        return self.check_ids(roots, targets)

    def close(self):
        if getattr(self, "h", None):
            self.L.ketogpu_part_engine_free(self.h)
            self.h = None
        close = getattr(self.local, "close", None)
        if close:
            close()

    def __del__(self):
        self.close()


class Core:
    """The core of a partitioned network on every rank (ketogpu_core_gather, collective):
    the rows among interior nodes — interior successors and interior predecessors of every
    interior node — gathered from their owners.  Raises KETOGPU_ENOMEM on every rank alike
    when it passes `budget` bytes of device records (then use PartitionedEngine)."""

    def __init__(self, shard, comm=None, budget=0):
        self.L = L.lib()
        self.shard = shard
        comm = comm if comm is not None else shard.native_comm()
        h = C.c_void_p()
        L.check(self.L.ketogpu_core_gather(shard.h, comm.handle, int(budget), C.byref(h)))
        self.h = h

    def view(self):
        v = L.CoreView()
        L.check(self.L.ketogpu_core_get_view(self.h, C.byref(v)))
        n = v.num_interior

        def arr(p, k, dt):
            return np.ctypeslib.as_array(p, (k,)).copy() if k else np.zeros(0, dtype=dt)
        f_off = arr(v.f_off, n + 1, np.uint64)
        b_off = arr(v.b_off, n + 1, np.uint64)
        return {"num_interior": n, "bytes": v.bytes, "f_off": f_off, "f_col": arr(v.f_col, int(f_off[-1]), np.uint32),
                "b_off": b_off, "b_col": arr(v.b_col, int(b_off[-1]), np.uint32)}

    def close(self):
        if getattr(self, "h", None):
            self.L.ketogpu_core_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


class TieredEngine:
    """check_ids over the partitioned graph in TWO exchanges per batch (ketogpu_tier_*,
    include/ketogpu.h "two-tier"): every rank holds the core (Core) and its own rows; a
    request's two seed rows travel from their owners, then the single-GPU engine's
    bidirectional LDS unit runs over the local core.  Unlike PartitionedEngine, each rank
    passes ITS OWN requests and gets their answers (the call is still collective: every
    rank calls check_ids once per batch, with 0 requests if it has none).  `local` (tests
    only): an object whose vtable() gives host steps (tests/tier_cpu.py)."""

    def __init__(self, shard, device=0, local=None, core=None, comm=None, max_batch=0, core_budget=0,
                 fallback_state_bytes=0):
        self.L = L.lib()
        self.shard = shard
        if comm is None:
            comm = shard.native_comm(device, host_steps=local is not None)
        self.ncomm = comm
        opts = L.TierOpts(device, int(max_batch), int(fallback_state_bytes))
        h = C.c_void_p()
        if local is None:
            self.core = core if core is not None else Core(shard, comm, core_budget)
            L.check(self.L.ketogpu_tier_new(shard.h, self.core.h, comm.handle, C.byref(opts), C.byref(h)))
            self.local = None
        else:
            self.core = core
            self.local = local
            self._vt = local.vtable()
            L.check(self.L.ketogpu_tier_new_steps(C.byref(self._vt), comm.handle, C.byref(opts), C.byref(h)))
        self.h = h

    def stats(self):
        st = L.TierStats()
        L.check(self.L.ketogpu_tier_stats_get(self.h, C.byref(st)))
        return st.as_dict()

    def check_ids(self, roots, targets):
        """this rank's (roots, targets) -> bool answers"""
        roots = np.ascontiguousarray(roots, dtype=np.uint32)
        targets = np.ascontiguousarray(targets, dtype=np.uint32)
        n = len(roots)
        bits = np.zeros(max((n + 63) // 64, 1), dtype=np.uint64)
        L.check(self.L.ketogpu_tier_check_ids(self.h, roots.ctypes.data, targets.ctypes.data, n, bits.ctypes.data))
        return np.unpackbits(bits.view(np.uint8), bitorder="little")[:n].astype(bool)

    def check_ids_ptr(self, roots_ptr, targets_ptr, n, bits):
        """the batch call on raw request pointers (host memory, or this device's HBM: read in
        place by every pass) -> bits (host uint64 array)"""
        L.check(self.L.ketogpu_tier_check_ids(self.h, roots_ptr, targets_ptr, n, bits.ctypes.data))

    def check_ids_raw(self, roots, targets, bits):
        """the batch call on caller arrays (pinned buffers are read in place at world 1)"""
        L.check(self.L.ketogpu_tier_check_ids(self.h, roots.ctypes.data, targets.ctypes.data, len(roots),
                                              bits.ctypes.data))

    def close(self):
        if getattr(self, "h", None):
            self.L.ketogpu_tier_free(self.h)
            self.h = None

    def __del__(self):
        self.close()
