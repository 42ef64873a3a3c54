"""Micro-batcher: concurrent SubjectIsAllowed calls coalesced into one engine batch.

SURVEY.md §8(b) "Threading" and "Cancellation": Keto calls the check engine from one
goroutine per HTTP/gRPC request (`internal/check/handler.go:95,134,154`), while the GPU
engine answers 64 requests per 64-bit word and amortises a launch over ~10^6 requests.
The batcher sits between the two, as the Go `batcher` sketched in INTEGRATION.md §2 would:

  * callers (any thread) `submit` one tuple and wait; a dispatcher thread flushes the
    queue as one `Engine.check_many` call when `max_batch` requests are waiting or the
    oldest has waited `max_wait` seconds;
  * a request whose context is cancelled before its batch is flushed is dropped from the
    batch; one cancelled while its batch runs gets `Canceled` and its result is discarded.
    Cancellation never fails the other requests of a batch;
  * a nil subject fails only its own request (`NilSubject`, the documented divergence from
    `internal/check/engine.go:46`), never the batch;
  * an engine failure (device error) fails exactly the requests of that batch, as each of
    those HTTP requests would get a 500 from the reference's error path.

`Context` is the minimal stand-in for Go's `context.Context` (cancel + deadline).
"""
import threading
import time
from concurrent.futures import Future
from concurrent.futures import TimeoutError as FutureTimeout  # builtin TimeoutError only from 3.11

from .relationtuple import InternalRelationTuple, NilSubject


class Canceled(Exception):
    """context.Canceled / context.DeadlineExceeded of the waiting caller"""


class Context:
    def __init__(self, timeout=None):
        self._ev = threading.Event()
        self.deadline = None if timeout is None else time.monotonic() + timeout

    def cancel(self):
        self._ev.set()

    def done(self):
        return self._ev.is_set() or (self.deadline is not None and time.monotonic() >= self.deadline)

    def remaining(self):
        return None if self.deadline is None else max(0.0, self.deadline - time.monotonic())


class MicroBatcher:
    def __init__(self, engine, max_batch=1 << 16, max_wait=200e-6):
        if max_batch < 1:
            raise ValueError("max_batch must be >= 1")
        self.engine = engine  # anything with check_many(list of tuples) -> list of bool
        self.max_batch = int(max_batch)
        self.max_wait = float(max_wait)
        self._cv = threading.Condition()
        self._queue = []  # (tuple, future, ctx, enqueue time)
        self._closed = False
        self.batches = []  # sizes of the flushed batches (diagnostics)
        self._thread = threading.Thread(target=self._run, name="keto-micro-batcher", daemon=True)
        self._thread.start()

    # ------------------------------------------------------------ callers
    def submit(self, r: InternalRelationTuple, ctx: Context = None) -> Future:
        f = Future()
        if r is None or r.subject is None:
            f.set_exception(NilSubject("subject is not allowed to be nil"))
            return f
        with self._cv:
            if self._closed:
                raise RuntimeError("batcher is closed")
            self._queue.append((r, f, ctx, time.monotonic()))
            if len(self._queue) >= self.max_batch or len(self._queue) == 1:
                self._cv.notify()
        return f

    def SubjectIsAllowed(self, r: InternalRelationTuple, ctx: Context = None) -> bool:
        """blocking form with the engine's signature; raises Canceled when ctx ends first"""
        f = self.submit(r, ctx)
        while True:
            wait = 0.01 if ctx is None or ctx.remaining() is None else min(0.01, ctx.remaining())
            try:
                return f.result(timeout=wait)
            except FutureTimeout:
                if ctx is not None and ctx.done():
                    raise Canceled("context canceled while the check was queued or running") from None

    subject_is_allowed = SubjectIsAllowed

    def check_many(self, tuples):
        """an explicit batch (POST /check/batch) is already a batch: straight to the engine"""
        return self.engine.check_many(tuples)

    def close(self):
        with self._cv:
            self._closed = True
            self._cv.notify()
        self._thread.join()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ------------------------------------------------------------ dispatcher
    def _take(self):
        """wait until a batch is due; returns it (empty list: closed and drained)"""
        with self._cv:
            while True:
                if self._queue:
                    age = time.monotonic() - self._queue[0][3]
                    if len(self._queue) >= self.max_batch or age >= self.max_wait or self._closed:
                        batch, self._queue = self._queue[:self.max_batch], self._queue[self.max_batch:]
                        return batch
                    self._cv.wait(self.max_wait - age)
                elif self._closed:
                    return []
                else:
                    self._cv.wait()

    @staticmethod
    def _settle(f, result=None, exc=None):
        """complete one request's future; a future its caller cancelled (Future.cancel) is
        skipped, so no single request can raise InvalidStateError in the dispatcher"""
        try:
            if exc is not None:
                f.set_exception(exc)
            else:
                f.set_result(result)
        except Exception:  # cancelled or already settled: that caller is gone
            pass

    def _run(self):
        while True:
            batch = self._take()
            if not batch:
                return
            try:
                self._dispatch(batch)
            except Exception as e:  # never let one batch end the dispatcher thread
                for _, f, _, _ in batch:
                    if not f.done():
                        self._settle(f, exc=e)

    def _dispatch(self, batch):
        live = []
        for item in batch:
            r, f, ctx, _ = item
            # claim the future first: set_running_or_notify_cancel() is False for a future the
            # caller already cancelled, which then takes no outcome at all
            if not f.set_running_or_notify_cancel():
                continue
            if ctx is not None and ctx.done():  # dropped before it reaches the device
                self._settle(f, exc=Canceled("context canceled before the batch was flushed"))
            else:
                live.append(item)
        if not live:
            return
        self.batches.append(len(live))
        try:
            got = self.engine.check_many([r for r, _, _, _ in live])
        except Exception as e:  # device failure: exactly this batch's requests fail
            for _, f, _, _ in live:
                self._settle(f, exc=e)
            return
        for (_, f, _, _), a in zip(live, got):
            self._settle(f, result=bool(a))
