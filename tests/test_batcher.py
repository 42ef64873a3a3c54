"""MicroBatcher (keto_amd/batcher.py): concurrent SubjectIsAllowed callers coalesced into
engine batches, with the cancellation and error isolation of SURVEY.md §8(b).  CPU tests
drive it with a stub engine whose answers come from the oracle; the GPU test uses the
real engine."""
import threading
import time

import numpy as np
import pytest

from keto_amd import relationtuple as rt
from keto_amd.batcher import Canceled, Context, MicroBatcher
from tests import randgraph


def tuples_of(reqs):
    return [rt.InternalRelationTuple(ns, o, r, rt.subject_from_dict(s)) for ns, o, r, s in reqs]


@pytest.fixture(scope="module")
def cases():
    namespaces, rows = randgraph.make_graph(71, n_rows=600, n_obj=30, n_users=40, poison=True)
    orc = randgraph.oracle_store(namespaces, rows, 5)
    reqs = randgraph.make_requests(71, namespaces, rows, n=800)
    want = [bool(x) for x in orc.check_batch(reqs)]
    return namespaces, rows, tuples_of(reqs), want


class StubEngine:
    """check_many answered from a table (the oracle's answers); optional gate to hold a batch"""

    def __init__(self, table, gate=None):
        self.table = table
        self.gate = gate
        self.seen = []
        self.entered = threading.Event()

    def check_many(self, tuples):
        self.seen.append([t.String() for t in tuples])
        self.entered.set()
        if self.gate is not None:
            self.gate.wait(10)
        return [self.table[t.String()] for t in tuples]


def table_of(tuples, want):
    return {t.String(): w for t, w in zip(tuples, want)}


def test_concurrent_callers_get_their_own_answers(cases):
    _, _, tuples, want = cases
    eng = StubEngine(table_of(tuples, want))
    got = [None] * len(tuples)
    with MicroBatcher(eng, max_batch=64, max_wait=2e-3) as b:
        def worker(k):
            for i in range(k, len(tuples), 16):
                got[i] = b.SubjectIsAllowed(tuples[i])
        ts = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert got == want
        assert max(b.batches) > 1 and max(b.batches) <= 64  # coalesced, bounded
        assert sum(b.batches) == len(tuples)


def test_futures_preserve_order_and_max_batch(cases):
    _, _, tuples, want = cases
    eng = StubEngine(table_of(tuples, want))
    with MicroBatcher(eng, max_batch=100, max_wait=0.05) as b:
        fs = [b.submit(t) for t in tuples]
        assert [f.result(5) for f in fs] == want
    assert all(len(s) <= 100 for s in eng.seen)


def test_cancelled_before_flush_is_dropped(cases):
    _, _, tuples, want = cases
    gate = threading.Event()
    eng = StubEngine(table_of(tuples, want), gate)
    with MicroBatcher(eng, max_batch=4, max_wait=1e-4) as b:
        f0 = b.submit(tuples[0])           # first batch: held inside the engine
        assert eng.entered.wait(5)
        ctx = Context()
        f1 = b.submit(tuples[1], ctx)      # queued behind the held batch
        f2 = b.submit(tuples[2])
        ctx.cancel()
        gate.set()
        assert f0.result(5) == want[0]
        with pytest.raises(Canceled):
            f1.result(5)
        assert f2.result(5) == want[2]
    assert all(tuples[1].String() not in s for s in eng.seen)  # never reached the device


def test_cancelled_while_running_does_not_fail_the_batch(cases):
    _, _, tuples, want = cases
    gate = threading.Event()
    eng = StubEngine(table_of(tuples, want), gate)
    with MicroBatcher(eng, max_batch=3, max_wait=10.0) as b:
        ctx = Context()
        out = {}

        def caller():
            try:
                out["a"] = b.SubjectIsAllowed(tuples[0], ctx)
            except Canceled as e:
                out["a"] = e
        th = threading.Thread(target=caller)
        th.start()
        time.sleep(0.05)
        f1, f2 = b.submit(tuples[1]), b.submit(tuples[2])  # a full batch of 3 flushes now
        assert eng.entered.wait(5)
        ctx.cancel()
        th.join(5)
        assert isinstance(out["a"], Canceled)
        gate.set()
        assert (f1.result(5), f2.result(5)) == (want[1], want[2])
    assert len(eng.seen) == 1 and len(eng.seen[0]) == 3


def test_deadline_cancels(cases):
    _, _, tuples, want = cases
    gate = threading.Event()
    eng = StubEngine(table_of(tuples, want), gate)
    with MicroBatcher(eng, max_batch=1, max_wait=0) as b:
        with pytest.raises(Canceled):
            b.SubjectIsAllowed(tuples[0], Context(timeout=0.05))
        gate.set()


def test_nil_subject_fails_alone(cases):
    _, _, tuples, want = cases
    eng = StubEngine(table_of(tuples, want))
    with MicroBatcher(eng, max_batch=8, max_wait=0.01) as b:
        bad = rt.InternalRelationTuple(tuples[0].namespace, tuples[0].object, tuples[0].relation, None)
        fb = b.submit(bad)
        fs = [b.submit(t) for t in tuples[:5]]
        with pytest.raises(rt.NilSubject):
            fb.result(5)
        assert [f.result(5) for f in fs] == want[:5]


def test_engine_failure_fails_only_its_batch(cases):
    _, _, tuples, want = cases

    class Flaky(StubEngine):
        def check_many(self, ts):
            if len(self.seen) == 0:
                self.seen.append(None)
                raise RuntimeError("device error")
            return super().check_many(ts)
    eng = Flaky(table_of(tuples, want))
    with MicroBatcher(eng, max_batch=4, max_wait=10.0) as b:
        first = [b.submit(t) for t in tuples[:4]]
        second = [b.submit(t) for t in tuples[4:8]]
        for f in first:
            with pytest.raises(RuntimeError):
                f.result(5)
        assert [f.result(5) for f in second] == want[4:8]


@pytest.mark.gpu
def test_batcher_on_gpu_engine(cases):
    from keto_amd import check
    from keto_amd.snapshot import Snapshot
    namespaces, rows, tuples, want = cases
    snap = Snapshot.from_rows(namespaces, rows, page_size=5, sort=True)
    eng = check.Engine(snap)
    got = [None] * len(tuples)
    with MicroBatcher(eng, max_batch=256, max_wait=1e-3) as b:
        def worker(k):
            for i in range(k, len(tuples), 8):
                got[i] = b.SubjectIsAllowed(tuples[i])
        ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    assert got == want
    assert np.mean(b.batches) > 1


def test_future_cancel_with_done_context_keeps_dispatcher(cases):
    """a caller that cancels its Future and its context must not kill the
    dispatcher (set_exception on a CANCELLED future raises InvalidStateError)"""
    _, _, tuples, want = cases
    gate = threading.Event()
    eng = StubEngine(table_of(tuples, want), gate=gate)
    with MicroBatcher(eng, max_batch=4, max_wait=1e-3) as b:
        first = b.submit(tuples[0])  # holds the dispatcher inside the engine call
        assert eng.entered.wait(5)
        ctx = Context()
        f = b.submit(tuples[1], ctx)
        assert f.cancel()  # still queued: the caller's cancel succeeds
        ctx.cancel()
        g = b.submit(tuples[2], Context())
        g.cancel()  # cancelled future, live context
        gate.set()
        assert first.result(5) == want[0]
        # the dispatcher is still alive and answers later requests
        assert b.SubjectIsAllowed(tuples[3]) == want[3]
        assert f.cancelled() and g.cancelled()
