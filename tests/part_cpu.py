"""CPU stand-in for one rank's device steps of the partitioned mode (TEST ONLY).

It implements the step interface of keto_amd.partition.DevicePartition in Python over the
rank's loaded shard (ketogpu_shard_view: its forward, reverse and backward rows in global
ids, and the id layout), with the same ownership arithmetic as partition.hip, so the
multi-rank exchange protocol of keto_amd.partition.PartitionedEngine runs for real over
gloo on CPU (world_size >= 2) without a GPU.  The product never uses it: the engine takes
it only when a test passes it in as `local`.
"""
from collections import defaultdict

import numpy as np

from keto_amd.partition import records_to_tensor, tensor_to_records

NONE = 0xFFFFFFFF


def owner(v, Ni, Nx, world):
    """partition.hip part_owner: ids interleave the ranks inside each class range"""
    v = np.asarray(v, dtype=np.int64)
    base = np.where(v < Ni, 0, np.where(v < Nx, Ni, Nx))
    return (v - base) % world


class CpuPartition:
    def __init__(self, view, words=4):
        self.v = view
        self.rank, self.world, self.words = view["rank"], view["world"], words
        self.Ni, self.Nx, self.N = view["num_interior"], view["num_expandable"], view["num_nodes"]

    def round_words(self):
        return self.words

    def owner(self, v):
        return owner(v, self.Ni, self.Nx, self.world)

    def local(self, v):
        """partition.hip p_local: the owned node's local index, or None"""
        v = int(v)
        if v >= self.N or int(self.owner(v)) != self.rank:
            return None
        w, g = self.world, self.v
        if v < self.Ni:
            l, lim = v // w, g["owned_interior"]
        elif v < self.Nx:
            l, lim = g["owned_interior"] + (v - self.Ni) // w, g["owned_expandable"]
        else:
            l, lim = g["owned_expandable"] + (v - self.Nx) // w, g["owned_nodes"]
        return l if l < lim else None

    def _rows(self, name, l):
        off, col = self.v[name + "_off"], self.v[name + "_col"]
        return [int(x) for x in col[off[l]:off[l + 1]]]

    def _fint(self, v):
        l = self.local(v)
        return self._rows("lf", l) if l is not None and l < self.v["owned_expandable"] else []

    def _rev(self, t):
        l = self.local(t)
        return self._rows("lr", l) if l is not None else []

    def _own(self, v):
        return self.local(v) is not None

    def _ipred(self, v):
        l = self.local(v)
        return self._rows("lb", l) if l is not None and l < self.v["owned_interior"] else []

    def _row(self, v):
        """the BFS row of v in the round's direction"""
        return self._ipred(v) if self.dir else self._fint(v)

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
                self.out += [(i >> 6, u, 1 << (i & 63)) for u in self._fint(r)]
            elif direction and self._own(t):  # backward: r in rev(t) is a hit, interior entries seed
                row = self._rev(t)
                if r in row:
                    self.hits.add(i)
                else:
                    self.out += [(i >> 6, v, 1 << (i & 63)) for v in row if v < self.Ni]
        return 0

    def _pack(self):
        out, self.out = self.out, []
        if not out:
            return 0, records_to_tensor([], [], []), [0] * self.world
        a = np.array([x[0] for x in out], dtype=np.uint32)
        b = np.array([x[1] for x in out], dtype=np.uint32)
        m = np.array([x[2] for x in out], dtype=np.uint64)
        dst = self.owner(b)
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
        return 0

    def pull_emit(self):
        for i, (r, t) in enumerate(zip(self.roots, self.targets)):
            if r == NONE or t == NONE or r >= self.Nx:
                continue
            if self.dir:  # backward: the root's owner asks whether u in fint(r) reaches t
                if self._own(r):
                    self.out += [(i, u, 0) for u in self._fint(r)]
                continue
            if not self._own(t):
                continue
            row = self._rev(t)
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
        return 0

    def end(self, n):
        bits = np.zeros(max((n + 63) // 64, 1), dtype=np.uint64)
        for i in self.hits:
            bits[i >> 6] |= np.uint64(1 << (i & 63))
        return bits

    def abort(self):
        self.out, self.nxt = [], {}
