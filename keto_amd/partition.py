"""Partitioned mode: batched checks over a hash-partitioned graph, one process per GPU.

BASELINE.json config #5 / SURVEY.md 8(e): when the snapshot does not fit one GPU, node v
is owned by rank ketogpu_part_owner(v, world) (= mix64(v) % world) and every rank holds
the rows and traversal state of its own nodes.  A round of up to 64*W requests is a
multi-source BFS whose levels exchange (word, node, mask) records between ranks:

    begin -> { emit -> all_to_all -> apply -> all_reduce(frontier) ; stop at 0 -> expand }
          -> pull_emit -> all_to_all -> pull_answer -> end -> all_reduce(MAX) of the hit bits

The device steps are libketogpu's ketogpu_part_* (keto_amd/csrc/partition.hip); this
module is the exchange: torch.distributed all_to_all_single on device tensors (backend
"nccl" = RCCL over xGMI), or through host memory for gloo.  It answers exactly what
check.Engine.check_ids answers (the same reachability formula, R2: no depth cutoff).
"""
import ctypes as C

import time

import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L

REC_COLS = 4  # a 16-byte ketogpu_record as 4 int32 columns


def records_to_tensor(a, b, m):
    """numpy (a u32, b u32, m u64) -> int32 tensor (n, 4) in ketogpu_record layout"""
    rec = np.empty(len(a), dtype=[("a", "<u4"), ("b", "<u4"), ("m", "<u8")])
    rec["a"], rec["b"], rec["m"] = a, b, m
    return torch.from_numpy(rec.view(np.int32).reshape(-1, REC_COLS).copy())


def tensor_to_records(t):
    """int32 tensor (n, 4) -> (a, b, m) numpy arrays"""
    rec = np.ascontiguousarray(t.cpu().numpy()).view([("a", "<u4"), ("b", "<u4"), ("m", "<u8")]).reshape(-1)
    return rec["a"].copy(), rec["b"].copy(), rec["m"].copy()


FORWARD, BACKWARD = 0, 1  # include/ketogpu.h KETOGPU_PART_FORWARD / _BACKWARD


class DevicePartition:
    """One rank's device steps (ketogpu_part_*); records travel in int32 tensors on its GPU."""

    def __init__(self, snapshot, rank, world, device=0, record_capacity=1 << 22, max_words_per_round=0,
                 state_budget_bytes=0):
        self.L = L.lib()
        self.snapshot = snapshot  # keeps the host snapshot alive
        self.world = world
        self.device = torch.device("cuda", device)
        opts = L.PartOpts(device, rank, world, record_capacity, max_words_per_round, state_budget_bytes)
        h = C.c_void_p()
        L.check(self.L.ketogpu_part_new(snapshot.h, C.byref(opts), C.byref(h)))
        self.h = h
        self.cap = record_capacity
        self.send = torch.empty((self.cap, REC_COLS), dtype=torch.int32, device=self.device)
        self.counts = np.zeros(max(world, 1), dtype=np.uint64)
        self._req = None

    def round_words(self):
        return int(self.L.ketogpu_part_round_words(self.h))

    def begin(self, roots, targets, direction=FORWARD):
        self._req = (np.ascontiguousarray(roots, dtype=np.uint32), np.ascontiguousarray(targets, dtype=np.uint32))
        r, t = self._req
        L.check(self.L.ketogpu_part_begin_dir(self.h, r.ctypes.data, t.ctypes.data, len(r), direction))

    def _pack(self, fn):
        rc = fn(self.h, self.send.data_ptr(), self.cap, self.counts.ctypes.data)
        if rc == L.ENOMEM:
            return 1, self.send[:0], [0] * self.world
        L.check(rc)
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
        rc = self.L.ketogpu_part_apply(self.h, recv.data_ptr() if len(recv) else None, len(recv), C.byref(fr))
        if rc == L.ENOMEM:
            return 1, 0
        L.check(rc)
        return 0, fr.value

    def expand(self):
        L.check(self.L.ketogpu_part_expand(self.h))

    def pull_answer(self, recv):
        recv = self._recv(recv)
        L.check(self.L.ketogpu_part_pull_answer(self.h, recv.data_ptr() if len(recv) else None, len(recv)))

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

    def close(self):
        if getattr(self, "h", None):
            self.L.ketogpu_part_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


class PartitionedEngine:
    """check_ids over the partitioned graph.  Every rank calls check_ids with the same
    (roots, targets) and gets the full answer.  `local` is the rank's step implementation
    (DevicePartition by default)."""

    def __init__(self, snapshot, device=0, group=None, local=None, direction="auto", **opts):
        """direction: "forward" (grow the roots' closures), "backward" (grow the targets'
        ancestor sets) or "auto": the first two full rounds run one direction each, timed
        (max over ranks, so every rank decides alike), and the faster is kept"""
        if direction not in ("auto", "forward", "backward"):
            raise ValueError("direction must be auto, forward or backward")
        self.direction = {"forward": FORWARD, "backward": BACKWARD}.get(direction)
        self._trial = {}  # direction -> ns per request of its trial round
        self._per = {FORWARD: 1 << 62, BACKWARD: 1 << 62}  # requests per round after overflow retries
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
            self.comm_cuda = dist.get_backend(group) == "nccl"
        else:
            self.rank, self.world, self.comm_cuda = 0, 1, False
        self.local = local if local is not None else DevicePartition(snapshot, self.rank, self.world, device, **opts)
        self.levels = 0
        self.retries = 0
        self.records = 0

    # ---------------------------------------------------------------- collectives
    def _comm_device(self):
        return torch.device("cuda", torch.cuda.current_device()) if self.comm_cuda else torch.device("cpu")

    def _allreduce(self, vals, op):
        if self.world == 1:
            return [int(v) for v in vals]
        t = torch.tensor(vals, dtype=torch.int64, device=self._comm_device())
        dist.all_reduce(t, op=op, group=self.group)
        return [int(v) for v in t.tolist()]

    def _alltoall(self, send, counts):
        self.records += int(sum(counts))
        if self.world == 1:
            return send
        cdev = self._comm_device()
        cnt = torch.tensor(counts, dtype=torch.int64, device=cdev)
        rcnt = torch.empty_like(cnt)
        dist.all_to_all_single(rcnt, cnt, group=self.group)
        rc = [int(x) for x in rcnt.tolist()]
        recv = torch.empty((sum(rc), REC_COLS), dtype=torch.int32, device=cdev)
        dist.all_to_all_single(recv, send.to(cdev), rc, list(counts), group=self.group)
        return recv

    # -------------------------------------------------------------------- rounds
    def _round(self, roots, targets, direction):
        """one round; None when a rank's buffers overflowed (every rank aborts)"""
        loc = self.local
        loc.begin(roots, targets, direction)
        while True:
            st, send, counts = loc.emit()
            if self._allreduce([st], dist.ReduceOp.MAX if self.world > 1 else None)[0]:
                loc.abort()
                return None
            recv = self._alltoall(send, counts)
            st, frontier = loc.apply(recv)
            total, err = self._allreduce([frontier, st], dist.ReduceOp.SUM if self.world > 1 else None)
            if err:
                loc.abort()
                return None
            self.levels += 1
            if total == 0:  # no rank has a frontier left: the closure is complete
                break
            loc.expand()
        st, send, counts = loc.pull_emit()
        if self._allreduce([st], dist.ReduceOp.MAX if self.world > 1 else None)[0]:
            loc.abort()
            return None
        loc.pull_answer(self._alltoall(send, counts))
        bits = loc.end(len(roots))
        hit = np.unpackbits(bits.view(np.uint8), bitorder="little")[:len(roots)]
        if self.world > 1:  # the answer is the OR of the ranks' hits
            t = torch.from_numpy(hit.copy()).to(self._comm_device())
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            hit = t.cpu().numpy()
        return hit.astype(bool)

    def check_ids(self, roots, targets):
        roots = np.ascontiguousarray(roots, dtype=np.uint32)
        targets = np.ascontiguousarray(targets, dtype=np.uint32)
        n = len(roots)
        top = self._allreduce([self.local.round_words() * 64], dist.ReduceOp.MIN if self.world > 1 else None)[0]
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
                    self._trial[d] = self._allreduce([ns], dist.ReduceOp.MAX if self.world > 1 else None)[0]
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

    def _shrink(self, d, m):
        if m <= 64:
            raise L.KetoError(L.ENOMEM, "partition buffers overflow for a single 64-request word")
        self._per[d] = max(64, (m // 2) // 64 * 64)
        self.retries += 1

    def close(self):
        close = getattr(self.local, "close", None)
        if close:
            close()
