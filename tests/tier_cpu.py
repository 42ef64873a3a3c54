"""CPU stand-in for one rank's device steps of the two-tier partitioned mode (TEST ONLY).

It implements include/ketogpu.h ketogpu_tier_steps (queries / reply_sizes / reply_emit /
evaluate) in Python over the rank's loaded shard (ketogpu_shard_view) and the gathered core
(ketogpu_core_get_view), with the ownership arithmetic of device_engine.hip tier_local /
tier_owner, so the NATIVE protocol (ketogpu_tier_check_ids, keto_amd/csrc/tier.cpp) and its
collectives run for real over gloo on CPU (world_size >= 2) without a GPU.  Its evaluation
is the R2 formula written plainly: allowed(r, t) <=> r in rev(t) or rev(t) meets
X(r), X(r) the interior closure of fint(r) over the core's forward rows.  The product never
uses it: keto_amd.partition.TieredEngine takes it only when a test passes it as `local`.
"""
import ctypes as C
from collections import defaultdict

import numpy as np

from keto_amd import _lib as L
from tests.part_cpu import NONE, owner

QUERY = np.dtype([("tag", "<u4"), ("node", "<u4")])                                  # ketogpu_tier_query
REC = np.dtype([("node", "<u4"), ("tag", "<u4")])  # ketogpu_tier_rec


class CpuTier:
    def __init__(self, view, core):
        self.v, self.core = view, core
        self.rank, self.world = view["rank"], view["world"]
        self.Ni, self.Nx, self.N = view["num_interior"], view["num_expandable"], view["num_nodes"]
        self.calls = defaultdict(int)
        self.pending = None

    def owner(self, v):
        return owner(v, self.Ni, self.Nx, self.world)

    def local(self, v):
        v, w, g = int(v), self.world, self.v
        if v >= self.N or int(self.owner(v)) != self.rank:
            return None
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

    def _row(self, node, d):
        """the seed row a query asks for: fint(node) (d = 0) or rev(node) (d = 1)"""
        l = self.local(node)
        assert l is not None, "query routed to the wrong rank"
        if d:
            return self._rows("lr", l)
        return self._rows("lf", l) if l < self.v["owned_expandable"] else []

    def _core_row(self, u):
        off, col = self.core["f_off"], self.core["f_col"]
        return col[off[u]:off[u + 1]]

    # ------------------------------------------------------------------ steps
    def queries(self, roots, targets, send, counts):
        out = []
        for i, (r, t) in enumerate(zip(roots, targets)):
            r, t = int(r), int(t)
            if r == NONE or t == NONE or r >= self.Nx or t >= self.N:
                continue
            out += [(i << 1, r), (i << 1 | 1, t)]
        q = np.array(out, dtype=QUERY) if out else np.zeros(0, dtype=QUERY)
        dst = self.owner(q["node"]) if len(q) else np.zeros(0, dtype=np.int64)
        q = q[np.argsort(dst, kind="stable")]
        c = np.bincount(dst, minlength=self.world) if len(q) else np.zeros(self.world, dtype=np.int64)
        if len(q):
            C.memmove(send, q.tobytes(), q.nbytes)
        for g in range(self.world):
            counts[g] = int(c[g])
        return 0

    def reply_sizes(self, recv, n, frm, counts):
        q = np.frombuffer(C.string_at(recv, n * QUERY.itemsize), dtype=QUERY) if n else np.zeros(0, dtype=QUERY)
        recs, at = [], 0
        for p in range(self.world):
            k = 0
            for tag, node in q[at:at + int(frm[p])].tolist():
                row = self._row(node, tag & 1)
                recs += [(x, tag) for x in row]
                k += len(row)
            counts[p] = k
            at += int(frm[p])
        self.pending = np.array(recs, dtype=REC) if recs else np.zeros(0, dtype=REC)
        return 0

    def reply_emit(self, send):
        if len(self.pending):
            C.memmove(send, self.pending.tobytes(), self.pending.nbytes)
        return 0

    def evaluate(self, roots, targets, recv, nrecv, bits):
        fint, rev = defaultdict(list), defaultdict(list)
        n = len(roots)
        if recv is None:  # world 1: the rank's own rows
            for i in range(n):
                r, t = int(roots[i]), int(targets[i])
                if r != NONE and t != NONE and r < self.Nx and t < self.N:
                    fint[i], rev[i] = self._row(r, 0), self._row(t, 1)
        else:
            for node, tag in recv.tolist():
                (rev if tag & 1 else fint)[tag >> 1].append(node)
        for i in range(n):
            r, t = int(roots[i]), int(targets[i])
            if (r != NONE and r >= self.Nx) or (t != NONE and t >= self.N):
                return L.EINVAL
            if r == NONE or t == NONE:
                continue
            pred = set(rev[i])
            if r in pred:
                bits[i >> 6] |= 1 << (i & 63)
                continue
            seen, todo = set(), list(fint[i])
            while todo:
                u = todo.pop()
                if u in seen:
                    continue
                seen.add(u)
                if u in pred:
                    bits[i >> 6] |= 1 << (i & 63)
                    break
                todo += [int(x) for x in self._core_row(u)]
        return 0

    # ------------------------------------------------------ the C steps vtable
    def vtable(self):
        """include/ketogpu.h ketogpu_tier_steps over this object"""
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

        def arr(p, n):
            return np.ctypeslib.as_array(p, (n,)).copy() if n else np.zeros(0, dtype=np.uint32)

        def queries(_c, roots, targets, n, send, counts):
            return self.queries(arr(roots, n), arr(targets, n), send, counts)

        def evaluate(_c, roots, targets, n, recv, nrecv, bits, overflow, n_over):
            n_over[0] = 0
            rec = None
            if recv:
                rec = np.frombuffer(C.string_at(recv, nrecv * REC.itemsize), dtype=REC) if nrecv else \
                    np.zeros(0, dtype=REC)
            words = np.zeros(max((n + 63) // 64, 1), dtype=object)
            words[:] = 0
            code = self.evaluate(arr(roots, n), arr(targets, n), rec, nrecv, words)
            for k in range((n + 63) // 64):
                bits[k] = int(words[k])
            return code

        self._fns = (L.TIER_QUERIES_FN(guard("queries", queries)),
                     L.TIER_REPLY_SIZES_FN(guard("reply_sizes", lambda _c, recv, n, frm, counts:
                                                 self.reply_sizes(recv, n, frm, counts))),
                     L.TIER_REPLY_EMIT_FN(guard("reply_emit", lambda _c, send: self.reply_emit(send))),
                     L.TIER_EVALUATE_FN(guard("evaluate", evaluate)))
        return L.TierSteps(None, *self._fns)
