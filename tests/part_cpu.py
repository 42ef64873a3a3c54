"""CPU stand-in for one rank's device steps of the partitioned mode (TEST ONLY).

It implements the step interface of keto_amd.partition.DevicePartition in numpy over the
snapshot's device graph (ketogpu_snapshot_graph), with the same ownership function, so
the multi-rank exchange protocol of keto_amd.partition.PartitionedEngine runs for real
over gloo on CPU (world_size >= 2) without a GPU.  The product never uses it: the engine
takes it only when a test passes it in as `local`.
"""
from collections import defaultdict

import numpy as np

from keto_amd.partition import records_to_tensor, tensor_to_records

NONE = 0xFFFFFFFF


def owner(v, world):
    """mix64(v) % world, as ketogpu_part_owner"""
    x = np.asarray(v, dtype=np.uint64).copy()
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    return (x % np.uint64(world)).astype(np.int64)


class CpuPartition:
    def __init__(self, graph, rank, world, words=4):
        self.g = graph
        self.rank, self.world, self.words = rank, world, words
        self.Ni, self.Nx = graph["Ni"], graph["Nx"]

    def round_words(self):
        return self.words

    def _fint(self, v):
        fo = self.g["fint_off"]
        return self.g["fint_col"][fo[v]:fo[v + 1]]

    def _rev(self, t):
        ro = self.g["rev_off"]
        return self.g["rev_col"][ro[t]:ro[t + 1]]

    def _own(self, v):
        return int(owner(v, self.world)) == self.rank

    def _ipred(self, v):
        return [int(p) for p in self._rev(v) if p < self.Ni]

    def _row(self, v):
        """the BFS row of v in the round's direction"""
        return self._ipred(v) if self.dir else [int(u) for u in self._fint(v)]

    def begin(self, roots, targets, direction=0):
        self.roots, self.targets = [int(x) for x in roots], [int(x) for x in targets]
        self.dir = direction
        self.vis = defaultdict(int)
        self.nxt = {}
        self.hits = set()
        self.out = []
        for i, (r, t) in enumerate(zip(self.roots, self.targets)):
            if r == NONE or t == NONE or r >= self.Nx:
                continue
            if not direction and self._own(r):  # forward: seeds from the root's row
                self.out += [(i >> 6, int(u), 1 << (i & 63)) for u in self._fint(r)]
            elif direction and self._own(t):  # backward: r in rev(t) is a hit, interior entries seed
                row = [int(x) for x in self._rev(t)]
                if r in row:
                    self.hits.add(i)
                else:
                    self.out += [(i >> 6, v, 1 << (i & 63)) for v in row if v < self.Ni]

    def _pack(self):
        out, self.out = self.out, []
        if not out:
            return 0, records_to_tensor([], [], []), [0] * self.world
        a = np.array([x[0] for x in out], dtype=np.uint32)
        b = np.array([x[1] for x in out], dtype=np.uint32)
        m = np.array([x[2] for x in out], dtype=np.uint64)
        dst = owner(b, self.world)
        order = np.argsort(dst, kind="stable")
        counts = np.bincount(dst, minlength=self.world).tolist()
        return 0, records_to_tensor(a[order], b[order], m[order]), counts

    def emit(self):
        return self._pack()

    def apply(self, recv):
        a, b, m = tensor_to_records(recv)
        for w, v, mask in zip(a.tolist(), b.tolist(), m.tolist()):
            assert self._own(v) and v < self.Ni, "record routed to the wrong rank"
            new = mask & ~self.vis[(w, v)]
            if new:
                self.vis[(w, v)] |= new
                if len(self._row(v)):
                    self.nxt[(w, v)] = self.nxt.get((w, v), 0) | new
        return 0, len(self.nxt)

    def expand(self):
        nxt, self.nxt = self.nxt, {}
        for (w, v), mask in nxt.items():
            self.out += [(w, u, mask) for u in self._row(v)]

    def pull_emit(self):
        for i, (r, t) in enumerate(zip(self.roots, self.targets)):
            if r == NONE or t == NONE or r >= self.Nx:
                continue
            if self.dir:  # backward: the root's owner asks whether u in fint(r) reaches t
                if self._own(r):
                    self.out += [(i, int(u), 0) for u in self._fint(r)]
                continue
            if not self._own(t):
                continue
            row = [int(x) for x in self._rev(t)]
            if r in row:
                self.hits.add(i)
                continue
            self.out += [(i, v, 0) for v in row if v < self.Ni]
        return self._pack()

    def pull_answer(self, recv):
        a, b, _ = tensor_to_records(recv)
        for i, v in zip(a.tolist(), b.tolist()):
            assert self._own(v)
            if (self.vis.get((i >> 6, v), 0) >> (i & 63)) & 1:
                self.hits.add(i)

    def end(self, n):
        bits = np.zeros(max((n + 63) // 64, 1), dtype=np.uint64)
        for i in self.hits:
            bits[i >> 6] |= np.uint64(1 << (i & 63))
        return bits

    def abort(self):
        self.out, self.nxt = [], {}
