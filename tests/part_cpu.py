"""CPU stand-in for one rank's device steps of the partitioned mode (TEST ONLY).

It implements the steps of include/ketogpu.h ketogpu_part_steps (the ketogpu_part_begin_dir
/ _emit / _pull_emit / _apply / _expand / _pull_answer / _end / _abort sequence) in Python
over the rank's loaded shard (ketogpu_shard_view: its forward, reverse and backward rows in
global ids, and the id layout), with the same ownership arithmetic as partition.hip, so the
NATIVE round driver (ketogpu_part_check_ids, keto_amd/csrc/part_round.cpp) and its
collectives run for real over gloo on CPU (world_size >= 2) without a GPU.  The product
never uses it: keto_amd.partition.PartitionedEngine takes it only when a test passes it in
as `local` (its vtable() hands the callbacks to ketogpu_part_engine_new_steps).
"""
import ctypes as C
from collections import defaultdict

import numpy as np

from keto_amd import _lib as L

NONE = 0xFFFFFFFF
REC = np.dtype([("a", "<u4"), ("b", "<u4"), ("m", "<u8")])  # ketogpu_record


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
        self.out = []
        self.calls = defaultdict(int)

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

    # ------------------------------------------------------------------ steps
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

    def _pack(self, send, cap, counts):
        """this step's records grouped by destination into the library's buffer"""
        out, self.out = self.out, []
        c = np.zeros(self.world, dtype=np.int64)
        if out:
            rec = np.array(out, dtype=REC)
            dst = self.owner(rec["b"])
            rec = rec[np.argsort(dst, kind="stable")]
            c = np.bincount(dst, minlength=self.world)
            if len(rec) > cap:
                return L.ENOMEM
            C.memmove(send, rec.tobytes(), rec.nbytes)
        for g in range(self.world):
            counts[g] = int(c[g])
        return 0

    def emit(self, pull, send, cap, counts):
        if pull:
            self.pull_emit()
        return self._pack(send, cap, counts)

    def _records(self, recv, n):
        return np.frombuffer(C.string_at(recv, n * REC.itemsize), dtype=REC) if n else np.zeros(0, dtype=REC)

    def apply(self, recv, n, frontier):
        for w, v, mask in self._records(recv, n).tolist():
            assert self._own(v) and v < self.Ni, "record routed to the wrong rank"
            new = mask & ~self.vis[(w, v)]
            if new:
                self.vis[(w, v)] |= new
                if len(self._row(v)):
                    self.nxt[(w, v)] = self.nxt.get((w, v), 0) | new
        frontier[0] = len(self.nxt)
        return 0

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

    def pull_answer(self, recv, n):
        for i, v, _ in self._records(recv, n).tolist():
            assert self._own(v)
            if (self.vis.get((i >> 6, v), 0) >> (i & 63)) & 1:
                self.hits.add(i)
        return 0

    def end(self, bits):
        for i in self.hits:
            bits[i >> 6] |= 1 << (i & 63)
        return 0

    def abort(self):
        self.out, self.nxt = [], {}
        return 0

    # ------------------------------------------------------ the C steps vtable
    def vtable(self):
        """include/ketogpu.h ketogpu_part_steps over this object; an exception in a step is
        re-raised by the test after the library reports the failed call"""
        self.error = None

        def guard(name, fn):
            def run(*a):
                self.calls[name] += 1
                try:
                    return fn(*a)
                except Exception as e:  # noqa: BLE001 - surfaced through the status code
                    self.error = e
                    return L.EDEVICE
            return run

        def begin(_ctx, roots, targets, n, d):
            return self.begin(np.ctypeslib.as_array(roots, (n,)) if n else [],
                              np.ctypeslib.as_array(targets, (n,)) if n else [], d)

        self._fns = (L.BEGIN_FN(guard("begin", begin)),
                     L.EMIT_FN(guard("emit", lambda _c, pull, send, cap, counts: self.emit(pull, send, cap, counts))),
                     L.APPLY_FN(guard("apply", lambda _c, recv, n, fr: self.apply(recv, n, fr))),
                     L.STEP_FN(guard("expand", lambda _c: self.expand())),
                     L.PULL_ANSWER_FN(guard("pull_answer", lambda _c, recv, n: self.pull_answer(recv, n))),
                     L.END_FN(guard("end", lambda _c, bits: self.end(bits))),
                     L.STEP_FN(guard("abort", lambda _c: self.abort())))
        return L.PartSteps(None, self.words, *self._fns)
