"""Host-to-host batches (ketogpu_check_ids: chunked upload overlapped with the traversal,
device-side id validation) and the replicated multi-GPU engine (ketogpu_multi_*).

CPU: the range split of ketogpu_multi_range and the failure without a device.  GPU: every
path against the oracle (bit-exact), the pipelined first stage against the HBM-resident
run, pinned and pageable host arrays, ids outside the snapshot, requests that spill to the
global path inside a pipelined call."""
import numpy as np
import pytest

from keto_amd import _lib as L
from keto_amd import check, synth
from keto_amd import relationtuple as rt
from keto_amd.snapshot import Snapshot
from tests import randgraph


@pytest.mark.parametrize("n,parts", [(0, 1), (1, 1), (63, 2), (64, 2), (1000, 3), (10, 4), (1 << 20, 8),
                                     (1_000_001, 7)])
def test_multi_ranges_are_word_aligned_and_cover_the_batch(n, parts):
    r = check.MultiEngine.ranges(n, parts)
    assert len(r) == parts
    assert r[0][0] == 0 and r[-1][1] == n
    for (b0, e0), (b1, e1) in zip(r, r[1:]):
        assert e0 == b1  # contiguous
    words = [((e + 63) // 64 - b // 64) if e > b else 0 for b, e in r]
    for b, e in r:
        assert b % 64 == 0 or b == n  # every range starts on a result word
    assert max(words) - min(words) <= 1  # balanced to one word


def test_multi_engine_without_device_fails_cleanly():
    if L.lib().ketogpu_device_count() > 0:
        pytest.skip("a HIP device is visible")
    snap = Snapshot.from_rows([("n", 1)], [(1, "o", "r", "u", None, None, None)])
    with pytest.raises(L.KetoError) as e:
        check.MultiEngine(snap, [0])
    assert e.value.code == L.EDEVICE


@pytest.fixture(scope="module")
def rbac():
    w = synth.rbac(users=20000, groups=2000, docs=4000, tuples=120000, checks=70000, seed=21)
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    roots, targets = w.resolve(snap)
    want = randgraph.oracle_store_columns(w.namespaces, w.columns).check_batch(
        w.requests(range(len(roots))), nthreads=8)
    return w, snap, roots, targets, np.asarray(want, dtype=bool)


def _gpu():
    if L.lib().ketogpu_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")


def _pipe_mode(monkeypatch, mode):
    """direct[K]: pinned requests read in place by one launch, K units per workgroup;
    chunks: the chunk pipeline"""
    monkeypatch.setenv("KETOGPU_PIPE_MODE", "chunks" if mode == "chunks" else "direct")
    if mode.startswith("direct") and mode != "direct":
        monkeypatch.setenv("KETOGPU_HOST_UNITS", mode[len("direct"):])


@pytest.mark.gpu
@pytest.mark.parametrize("plan", ["bidi", "lite", "lite32", "core", "label"])
@pytest.mark.parametrize("mode", ["direct", "direct1", "direct4", "chunks"])
@pytest.mark.parametrize("chunk", ["4096", "65536", "1048576"])
def test_pipelined_check_ids_matches_oracle(rbac, chunk, mode, plan, monkeypatch):
    """bidi and lite plans, host batches: pinned requests read in place by one first-stage
    launch (direct) or by the chunk pipeline (several chunk sizes: many chunks, a few, one =
    not pipelined), and pageable host arrays; the HBM-resident run agrees"""
    _gpu()
    _, snap, roots, targets, want = rbac
    monkeypatch.setenv("KETOGPU_UNITS", plan)
    monkeypatch.setenv("KETOGPU_PIPE_CHUNK", chunk)
    _pipe_mode(monkeypatch, mode)
    eng = check.Engine(snap)
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
    pr, pt = check.pinned(roots), check.pinned(targets)
    words = (len(roots) + 63) // 64
    out = check.PinnedBuffer(words, np.uint64)
    for _ in range(3):  # repeated calls reuse the engine's buffers
        out.array[:] = 0
        eng.check_ids_raw(pr.array.ctypes.data, pt.array.ctypes.data, len(roots), out.array.ctypes.data)
        np.testing.assert_array_equal(check.unpack_bits(out.array.copy(), len(roots)), want)
    q = eng.upload(roots, targets)
    q.run()
    np.testing.assert_array_equal(q.download(), want)
    # a smaller batch after a larger one (persistent buffers, stale words beyond n)
    np.testing.assert_array_equal(eng.check_ids(roots[:1000], targets[:1000]), want[:1000])


@pytest.mark.gpu
@pytest.mark.parametrize("plan", ["bidi", "label"])
@pytest.mark.parametrize("mode", ["direct", "direct4", "chunks"])
def test_check_ids_rejects_ids_outside_the_snapshot(rbac, mode, plan, monkeypatch):
    _gpu()
    _, snap, roots, targets, want = rbac
    monkeypatch.setenv("KETOGPU_UNITS", plan)
    monkeypatch.setenv("KETOGPU_PIPE_CHUNK", "4096")
    _pipe_mode(monkeypatch, mode)
    eng = check.Engine(snap)
    st = snap.stats()
    words = (len(roots) + 63) // 64
    out = check.PinnedBuffer(words, np.uint64)
    for bad_at, which in ((0, "root"), (5000, "target"), (len(roots) - 1, "root")):
        r, t = roots.copy(), targets.copy()
        if which == "root":
            r[bad_at] = st["num_expandable"]  # not an expandable node
        else:
            t[bad_at] = st["num_nodes"] + 7
        with pytest.raises(L.KetoError) as e:
            eng.check_ids(r, t)
        assert e.value.code == L.EINVAL and f"request {bad_at} " in str(e.value)
        pr, pt = check.pinned(r), check.pinned(t)  # read in place by the device
        with pytest.raises(L.KetoError) as e:
            eng.check_ids_raw(pr.array.ctypes.data, pt.array.ctypes.data, len(r), out.array.ctypes.data)
        assert e.value.code == L.EINVAL and f"request {bad_at} " in str(e.value)
        with pytest.raises(L.KetoError):
            eng.upload(r, t)
    # the engine is still usable and exact afterwards, also for pinned batches read in place
    # back to back (plan label: a call after a clean call skips its clear launch), a smaller
    # batch after them and a larger one again
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
    pr, pt = check.pinned(roots), check.pinned(targets)
    for n in (len(roots), len(roots), 777, 64, len(roots)):
        out.array[:] = 0
        eng.check_ids_raw(pr.array.ctypes.data, pt.array.ctypes.data, n, out.array.ctypes.data)
        np.testing.assert_array_equal(check.unpack_bits(out.array.copy(), n), want[:n])


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["direct", "direct4", "chunks"])
def test_pipelined_call_with_global_path_spills(mode, monkeypatch):
    """a 20000-long chain of subject sets: requests whose search outgrows every LDS table
    (8192 slots at most) finish on the global path after the host-batch first stage"""
    _gpu()
    monkeypatch.setenv("KETOGPU_UNITS", "bidi")
    monkeypatch.setenv("KETOGPU_PIPE_CHUNK", "8192")
    _pipe_mode(monkeypatch, mode)
    n = 20000
    rows = [(1, f"g{i}", "m", None, 1, f"g{i + 1}", "m") for i in range(n)]
    rows.append((1, f"g{n}", "m", "alice", None, None, None))
    rows.append((1, "x", "m", "bob", None, None, None))
    snap = Snapshot.from_rows([("n", 1)], rows, sort=True)
    rng = np.random.default_rng(4)
    pos = rng.integers(0, n + 1, size=40000)
    who = rng.integers(0, 2, size=40000)  # alice (reachable from every g_i) or bob (never)
    reqs = [("n", f"g{i}", "m", rt.SubjectID("alice" if k == 0 else "bob")) for i, k in zip(pos, who)]
    roots, targets = snap.resolve_many(reqs)
    eng = check.Engine(snap)
    got = eng.check_ids(roots, targets)
    np.testing.assert_array_equal(got, who == 0)
    assert eng.last_stats()["spilled_requests"] > 0
    pr, pt = check.pinned(roots), check.pinned(targets)  # pinned: read in place (direct)
    out = check.PinnedBuffer((len(roots) + 63) // 64, np.uint64)
    eng.check_ids_raw(pr.array.ctypes.data, pt.array.ctypes.data, len(roots), out.array.ctypes.data)
    np.testing.assert_array_equal(check.unpack_bits(out.array.copy(), len(roots)), who == 0)
    assert eng.last_stats()["spilled_requests"] > 0


@pytest.mark.gpu
def test_spill_stage_grids_follow_the_previous_run(monkeypatch):
    """spill stages size their persistent grids from the previous run's spills: a run with
    no spills (smallest grids) followed by one where most units spill must still answer
    every request (the grids only change speed)"""
    _gpu()
    monkeypatch.setenv("KETOGPU_UNITS", "bidi")
    n = 3000  # chains of 3000 subject sets outgrow the 512-slot first-stage tables
    rows = [(1, f"g{i}", "m", None, 1, f"g{i + 1}", "m") for i in range(n)]
    rows.append((1, f"g{n}", "m", "alice", None, None, None))
    rows += [(1, f"s{i}", "m", f"u{i}", None, None, None) for i in range(2000)]
    snap = Snapshot.from_rows([("n", 1)], rows, sort=True)
    eng = check.Engine(snap)
    easy = [("n", f"s{i}", "m", rt.SubjectID(f"u{(i * 7) % 2000}")) for i in range(2000)]
    r, t = snap.resolve_many(easy)
    for _ in range(3):
        np.testing.assert_array_equal(eng.check_ids(r, t), [(i * 7) % 2000 == i for i in range(2000)])
    assert eng.last_stats()["spilled_units"] == 0
    rng = np.random.default_rng(5)
    pos = rng.integers(0, n + 1, size=8000)
    who = rng.integers(0, 2, size=8000)
    hard = [("n", f"g{i}", "m", rt.SubjectID("alice" if k == 0 else "u3")) for i, k in zip(pos, who)]
    r, t = snap.resolve_many(hard)
    np.testing.assert_array_equal(eng.check_ids(r, t), who == 0)
    assert eng.last_stats()["spilled_units"] > 100


@pytest.mark.gpu
def test_multi_engine_matches_oracle(rbac):
    """every visible device (at least the box's one), and the same device count split into
    ranges whose boundaries fall inside 16-request units of the other split"""
    _gpu()
    _, snap, roots, targets, want = rbac
    ndev = L.lib().ketogpu_device_count()
    m = check.MultiEngine(snap, list(range(ndev)))
    np.testing.assert_array_equal(m.check_ids(roots, targets), want)
    np.testing.assert_array_equal(m.check_ids(roots[:777], targets[:777]), want[:777])
    assert m.last_stats(0)["checks"] > 0
    with pytest.raises(L.KetoError) as e:
        check.MultiEngine(snap, [0, 0])
    assert e.value.code == L.EINVAL


@pytest.mark.gpu
def test_pinned_subrange_pointers_every_engine(rbac):
    """requests in ketogpu_host_alloc buffers (portable + mapped) passed as pointers into the
    middle of the allocation — at an odd request offset, so every device range starts
    inside it — through Engine and MultiEngine, against the oracle; each device reads
    through its own view of the buffer"""
    _gpu()
    _, snap, roots, targets, want = rbac
    off, n = 37, len(roots)
    pr, pt = check.PinnedBuffer(n + off + 5), check.PinnedBuffer(n + off + 5)
    pr.array[:] = 0xFFFFFFFF
    pt.array[:] = 0xFFFFFFFF
    pr.array[off:off + n], pt.array[off:off + n] = roots, targets
    words = (n + 63) // 64
    out = check.PinnedBuffer(words + 3, np.uint64)
    ndev = L.lib().ketogpu_device_count()
    engines = [check.Engine(snap), check.MultiEngine(snap, list(range(ndev)))]
    for eng in engines:
        for k in (0, 1, 2):  # a fresh registry view on the first call, cached after
            out.array[:] = 0
            eng.check_ids_raw(pr.p.value + 4 * off, pt.p.value + 4 * off, n, out.p.value + 8 * 3)
            np.testing.assert_array_equal(check.unpack_bits(out.array[3:3 + words].copy(), n), want)
            assert not out.array[:3].any()


@pytest.mark.gpu
def test_engines_freed_after_their_snapshot():
    """a garbage collector may finalise a snapshot before the engines over it (a reference
    cycle): engine teardown then skips the snapshot's reader registry instead of touching
    freed memory (Snapshot::ReaderLink)"""
    _gpu()
    w = synth.rbac(users=500, groups=50, docs=100, tuples=3000, checks=200, seed=5)
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    eng = check.Engine(snap)
    multi = check.MultiEngine(snap, [0])
    roots, targets = w.resolve(snap)
    eng.check_ids(roots, targets)
    multi.check_ids(roots, targets)
    snap.__del__()  # the snapshot goes first
    multi.close()
    eng.close()
