"""Partitioned mode (BASELINE config #5): the partition-aware loader
(ketogpu_shard_*) and the multi-rank exchange protocol of keto_amd.partition against the
oracle.

CPU tests load real shards (the C++ loader) with world_size 1, 2 and 3 over gloo and run
the check protocol with each rank's device steps played by tests/part_cpu.py; they also
pin the refusals (wildcard subject sets, rows out of order, shared String() keys, hash
collisions) and that a rank holds about 1/world of the graph.  The GPU tests run the HIP
steps (partition.hip) with world_size 1 and with two ranks sharing the box's GPU."""
import os
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from keto_amd import _lib as L
from keto_amd import persistence
from keto_amd.snapshot import Snapshot
from tests import randgraph

NS_SMALL = None


def _case(seed, n_rows=900, n_req=700):
    """a random network without wildcard subject sets (the partitioned engine refuses them)
    in the backend's row order, with poisoned pages"""
    namespaces, rows = randgraph.make_graph(seed, n_rows=n_rows, n_obj=40, n_users=60, poison=True, wildcard=False)
    rows = randgraph.backend_sorted(rows)
    reqs = randgraph.make_requests(seed, namespaces, rows, n=n_req, wildcard=False)
    return namespaces, rows, reqs


def _batches(rows, size=97):
    """the ordered read in batches (groups cross batch boundaries)"""
    return lambda: (persistence.columnar(rows[i:i + size]) for i in range(0, max(len(rows), 1), size))


def _want(namespaces, rows, reqs):
    return randgraph.oracle_store(namespaces, rows).check_batch(reqs).astype(bool)


def _load(namespaces, rows, **kw):
    from keto_amd.partition import Shard
    return Shard.load(namespaces, _batches(rows), **kw)


def test_single_rank_shard_matches_whole_graph_snapshot():
    namespaces, rows, _ = _case(60)
    sh = _load(namespaces, rows)
    snap = Snapshot.from_rows(namespaces, rows, sort=False).stats()
    st = sh.stats()
    assert st["num_interior"] == snap["num_interior"] and st["num_expandable"] == snap["num_expandable"]
    assert st["interior_forward_edges"] == snap["num_interior_edges"]
    assert st["reverse_edges"] == snap["num_rev_edges"]
    assert st["rows"] == len(rows) and st["bad_rows"] == snap["num_bad_rows"]


@pytest.mark.parametrize("direction", ["forward", "backward", "auto"])
def test_protocol_single_rank_cpu(direction):
    from keto_amd.partition import PartitionedEngine
    from tests.part_cpu import CpuPartition
    namespaces, rows, reqs = _case(61)
    sh = _load(namespaces, rows)
    eng = PartitionedEngine(sh, local=CpuPartition(sh.view(), words=3), direction=direction)
    got = eng.check_requests(persistence.request_columns(reqs))
    np.testing.assert_array_equal(got, _want(namespaces, rows, reqs))
    if direction == "auto":  # both directions ran a trial round, then one was kept
        assert set(eng._trial) == {0, 1} and eng.direction in (0, 1)


def test_refusals_single_rank():
    from keto_amd.partition import Shard
    ns = [("a", 1), ("a:b", 2)]
    ok = [(1, "o", "r", "u", None, None, None)]
    # a wildcard subject set (R5)
    with pytest.raises(L.KetoError, match="wildcard") as e:
        _load(ns, ok + [(1, "p", "r", None, 1, "", "r")])
    assert e.value.code == L.EINVAL
    # rows out of ORDER BY order: a group appears twice
    rows = [(1, "o", "r", "u1", None, None, None), (1, "p", "r", "u2", None, None, None),
            (1, "o", "r", "u3", None, None, None)]
    with pytest.raises(L.KetoError, match="ORDER BY"):
        Shard.load(ns, lambda: iter([persistence.columnar(rows)]))
    # R4: the subject id "a:b#c" and the subject set a:b#c share a String() key; so do the
    # sets (a, "b:x", r) and (a:b, "x", r)
    for extra in ([(1, "o", "r", "a:b#c", None, None, None), (1, "q", "r", None, 1, "b", "c")],
                  [(1, "q", "r", None, 1, "b:x", "r"), (1, "q", "s", None, 2, "x", "r")]):
        with pytest.raises(L.KetoError, match="String"):
            _load(ns, randgraph.backend_sorted(ok + extra))
    # ':' and '#' alone are not ambiguous
    _load(ns, randgraph.backend_sorted(ok + [(1, "q", "r", "x:y#z", None, None, None),
                                             (1, "q", "s", None, 1, "b:x", "r")]))


def test_hash_collisions_are_detected_and_retried(monkeypatch):
    """node hashes narrowed to 16 bits (test knob): collisions happen, every one is caught
    (the typed keys differ) and the load is retried with another salt until one is free;
    at 4 bits no salt is, and the load fails with KETOGPU_ECOLLISION"""
    from keto_amd.partition import PartitionedEngine, Shard
    from tests.part_cpu import CpuPartition
    namespaces, rows, reqs = _case(65, n_rows=600)
    monkeypatch.setenv("KETOGPU_SHARD_HASH_BITS", "16")
    _reload_lib(monkeypatch)
    sh = Shard.load(namespaces, _batches(rows), tries=40)
    eng = PartitionedEngine(sh, local=CpuPartition(sh.view(), words=4), direction="forward")
    np.testing.assert_array_equal(eng.check_requests(persistence.request_columns(reqs)),
                                  _want(namespaces, rows, reqs))
    monkeypatch.setenv("KETOGPU_SHARD_HASH_BITS", "4")
    _reload_lib(monkeypatch)
    with pytest.raises(L.KetoError) as e:
        Shard.load(namespaces, _batches(rows), tries=3)
    assert e.value.code == L.ECOLLISION


def _reload_lib(monkeypatch):
    """the hash-width knob is read once per process: load a private copy of the library"""
    import shutil
    d = tempfile.mkdtemp()
    p = os.path.join(d, "libketogpu.so")
    shutil.copy(L.LIB_PATH, p)
    monkeypatch.setattr(L, "LIB_PATH", p)
    monkeypatch.setattr(L, "_lib", None)


def _worker(rank, world, port, seed, out_dir, device_steps, direction="auto"):
    import resource

    import torch.distributed as dist
    from keto_amd.partition import PartitionedEngine
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        namespaces, rows, reqs = _case(seed)
        sh = _load(namespaces, rows)
        if device_steps:
            eng = PartitionedEngine(sh, device=0, record_capacity=4096, max_words_per_round=4, direction=direction)
        else:
            from tests.part_cpu import CpuPartition
            eng = PartitionedEngine(sh, local=CpuPartition(sh.view(), words=4), direction=direction)
        got = eng.check_requests(persistence.request_columns(reqs))
        st = sh.stats()
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), got)
        np.save(os.path.join(out_dir, f"records{rank}.npy"),
                np.array([eng.records, eng.levels, st["owned_nodes"], st["forward_edges"], st["reverse_edges"],
                          st["host_bytes"], resource.getrusage(resource.RUSAGE_SELF).ru_maxrss]))
        eng.close()
    finally:
        dist.destroy_process_group()


def _fail_worker(rank, world, port, out_dir):
    """rank 1's apply fails on its second call: every rank must raise (no rank is left
    waiting in a collective), and the next batch must be answered normally"""
    import torch.distributed as dist
    from keto_amd.partition import PartitionedEngine
    from tests.part_cpu import CpuPartition
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class Failing(CpuPartition):
        armed = True

        def apply(self, recv, n, frontier):
            if self.rank == 1 and self.armed and self.calls["apply"] == 2:
                self.armed = False
                return L.EINVAL
            return super().apply(recv, n, frontier)
    try:
        namespaces, rows, reqs = _case(67)
        sh = _load(namespaces, rows)
        eng = PartitionedEngine(sh, local=Failing(sh.view(), words=4), direction="forward")
        cols = persistence.request_columns(reqs)
        try:
            eng.check_requests(cols)
            code, msg = 0, ""
        except L.KetoError as e:
            code, msg = e.code, str(e)
        got = eng.check_requests(cols)
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), got)
        with open(os.path.join(out_dir, f"err{rank}.txt"), "w") as f:
            f.write(f"{code}\n{msg}")
    finally:
        dist.destroy_process_group()


def test_step_failure_on_one_rank_fails_every_rank():
    namespaces, rows, reqs = _case(67)
    want = _want(namespaces, rows, reqs)
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_fail_worker, args=(2, 29680, d), nprocs=2, join=True, start_method="spawn")
        errs = [open(os.path.join(d, f"err{r}.txt")).read().split("\n", 1) for r in range(2)]
        got = [np.load(os.path.join(d, f"rank{r}.npy")) for r in range(2)]
    assert [int(e[0]) for e in errs] == [L.EINVAL, L.EINVAL]
    assert "apply" in errs[1][1] and "another rank" in errs[0][1]
    for g in got:
        np.testing.assert_array_equal(g, want)


def _run_ranks(world, seed, device_steps, port, direction="auto"):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, port, seed, d, device_steps, direction), nprocs=world, join=True,
                           start_method="spawn")
        got = [np.load(os.path.join(d, f"rank{r}.npy")) for r in range(world)]
        rec = [np.load(os.path.join(d, f"records{r}.npy")) for r in range(world)]
    return got, rec


@pytest.mark.parametrize("world,seed,direction", [(2, 62, "forward"), (2, 62, "backward"), (3, 63, "auto")])
def test_protocol_multi_rank_gloo(world, seed, direction):
    namespaces, rows, reqs = _case(seed)
    want = _want(namespaces, rows, reqs)
    port = 29600 + world + 10 * ["forward", "backward", "auto"].index(direction)
    got, rec = _run_ranks(world, seed, device_steps=False, port=port, direction=direction)
    for g in got:  # every rank returns the full answer
        np.testing.assert_array_equal(g, want)
    assert all(r[0] > 0 for r in rec)  # records really crossed ranks
    assert want.any() and not want.all()
    # each rank owns a share of the nodes and rows, together the whole graph once
    single = _load(namespaces, rows).stats()
    assert sum(int(r[2]) for r in rec) == single["owned_nodes"]
    assert sum(int(r[3]) for r in rec) == single["forward_edges"]
    assert sum(int(r[4]) for r in rec) == single["reverse_edges"]
    assert max(int(r[2]) for r in rec) < single["owned_nodes"] * 0.75


def _c5_worker(rank, world, port, out_dir):
    import resource

    import torch.distributed as dist
    from keto_amd import synth
    from keto_amd.partition import PartitionedEngine, Shard
    from tests.part_cpu import CpuPartition
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = synth.config5(users=30000, groups=3000, docs=6000, tuples=150000, checks=1500, seed=17)
        sh = Shard.load(w.namespaces, lambda: w.batches(4093))
        roots, targets, st = sh.resolve_batch(w.request_batch())
        eng = PartitionedEngine(sh, local=CpuPartition(sh.view(), words=8), direction="backward")
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), eng.check_ids(roots, targets))
        np.save(os.path.join(out_dir, f"stats{rank}.npy"),
                np.array([sh.stats()["owned_nodes"], sh.stats()["host_bytes"],
                          resource.getrusage(resource.RUSAGE_SELF).ru_maxrss]))
    finally:
        dist.destroy_process_group()


def test_config5_stream_two_ranks_match_oracle():
    """the config #5 stream generator read by two ranks of the partition-aware loader, the
    check protocol over gloo, every answer against the oracle over the same stream"""
    from keto_amd import synth
    w = synth.config5(users=30000, groups=3000, docs=6000, tuples=150000, checks=1500, seed=17)
    from oracle import oracle as O
    st = O.Store(w.namespaces, 100)
    for cols in w.batches(4093):
        st.add_columnar(cols)
    want = st.finalize(presorted=True).check_batch(w.requests(range(w.n_checks)), nthreads=4)
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_c5_worker, args=(2, 29670, d), nprocs=2, join=True, start_method="spawn")
        got = [np.load(os.path.join(d, f"rank{r}.npy")) for r in range(2)]
        stats = [np.load(os.path.join(d, f"stats{r}.npy")) for r in range(2)]
    for g in got:
        np.testing.assert_array_equal(g, want)
    assert want[w.chk_pos.astype(bool)].all() and not want.all()
    assert all(s[0] > 0 for s in stats)


# --------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("direction", ["forward", "backward"])
@pytest.mark.parametrize("seed", [71, 72])
def test_partition_device_single_rank(seed, direction):
    from keto_amd.partition import PartitionedEngine
    if L.lib().ketogpu_device_count() < 1:
        pytest.fail("no HIP device visible")
    namespaces, rows, reqs = _case(seed, n_rows=1500, n_req=3000)
    sh = _load(namespaces, rows)
    want = _want(namespaces, rows, reqs)
    cols = persistence.request_columns(reqs)
    eng = PartitionedEngine(sh, device=0, max_words_per_round=8, direction=direction)
    np.testing.assert_array_equal(eng.check_requests(cols), want)
    st = eng.local.stats()
    assert st["rounds"] >= 6 and st["levels"] > 0 and st["records_sent"] > 0
    # tiny buffers: rounds overflow and are retried with fewer words, same answers
    small = PartitionedEngine(sh, device=0, record_capacity=2048, max_words_per_round=8, direction=direction)
    np.testing.assert_array_equal(small.check_requests(cols), want)
    assert small.retries > 0


@pytest.mark.gpu
def test_partition_device_rejects_ids_outside_the_snapshot():
    """an id outside the snapshot fails the round with KETOGPU_EINVAL (validated by the
    seed kernel), and the engine answers the next valid batch"""
    from keto_amd.partition import PartitionedEngine
    if L.lib().ketogpu_device_count() < 1:
        pytest.fail("no HIP device visible")
    namespaces, rows, reqs = _case(73, n_rows=800, n_req=500)
    sh = _load(namespaces, rows)
    want = _want(namespaces, rows, reqs)
    roots, targets, status = sh.resolve_batch(persistence.request_columns(reqs))
    eng = PartitionedEngine(sh, device=0, direction="backward")
    for bad_r, bad_t in ((1 << 30, 0), (0, 1 << 30)):
        r, t = roots.copy(), targets.copy()
        r[7], t[7] = (bad_r, t[7]) if bad_r else (r[7], bad_t)
        with pytest.raises(L.KetoError) as e:
            eng.check_ids(r, t)
        assert e.value.code == L.EINVAL
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)


@pytest.mark.gpu
def test_partition_device_rbac_matches_oracle():
    from keto_amd import check, synth
    from keto_amd.partition import PartitionedEngine, Shard
    w = synth.rbac(users=20000, groups=2000, docs=4000, tuples=120000, checks=20000, seed=9)
    sh = Shard.load(w.namespaces, lambda: iter([w.columns]))
    roots, targets, status = sh.resolve_batch(w.request_batch())
    assert not status.any()
    want = randgraph.oracle_store_columns(w.namespaces, w.columns).check_batch(
        w.requests(range(w.n_checks)), nthreads=8).astype(bool)
    for direction in ("forward", "backward"):
        np.testing.assert_array_equal(PartitionedEngine(sh, device=0, direction=direction).check_ids(roots, targets),
                                      want)
    eng = PartitionedEngine(sh, device=0, max_words_per_round=32)  # auto: trial rounds, then one direction
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
    assert set(eng._trial) == {0, 1}
    # the whole-graph engine agrees
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    np.testing.assert_array_equal(check.Engine(snap).check_ids(*w.resolve(snap)), want)


@pytest.mark.gpu
def test_partition_device_config5_matches_oracle():
    """BASELINE config #5's shape (synth.config5, streamed) at reduced size through the
    partition-aware loader and the HIP steps, every request against the oracle"""
    from keto_amd import synth
    from keto_amd.partition import PartitionedEngine, Shard
    w = synth.config5(users=100000, groups=10000, docs=40000, tuples=1_000_000, checks=20000, seed=23)
    from oracle import oracle as O
    st = O.Store(w.namespaces, 100)
    for cols in w.batches(1 << 16):
        st.add_columnar(cols)
    want = st.finalize(presorted=True).check_batch(w.requests(range(w.n_checks)), nthreads=8).astype(bool)
    sh = Shard.load(w.namespaces, lambda: w.batches(1 << 16))
    roots, targets, status = sh.resolve_batch(w.request_batch())
    for direction in ("forward", "backward", "auto"):
        eng = PartitionedEngine(sh, device=0, direction=direction)
        np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
    eng.local.set_timing(True)
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
    k = eng.local.stats()["kernels"]
    assert k["part_apply_kernel"]["launches"] > 0 and k["part_apply_kernel"]["ms"] > 0
    assert want[w.chk_pos.astype(bool)].all()


@pytest.mark.gpu
def test_partition_device_two_ranks_share_gpu():
    if L.lib().ketogpu_device_count() < 1:
        pytest.fail("no HIP device visible")
    namespaces, rows, reqs = _case(64)
    want = _want(namespaces, rows, reqs)
    got, rec = _run_ranks(2, 64, device_steps=True, port=29650)
    for g in got:
        np.testing.assert_array_equal(g, want)
    assert all(r[0] > 0 for r in rec)


def test_wildcard_root_is_refused_not_answered_false():
    """ketogpu_shard_resolve_batch marks a wildcard root (R5) ENOTFOUND; the
    reference can answer True there (the union of the groups it filters to), so the
    partitioned engine raises instead of answering False"""
    from keto_amd.partition import PartitionedEngine
    from tests.part_cpu import CpuPartition
    namespaces, rows, reqs = _case(66)
    sh = _load(namespaces, rows)
    eng = PartitionedEngine(sh, local=CpuPartition(sh.view(), words=3), direction="forward")
    ns, o, r, s = reqs[0]
    with pytest.raises(L.KetoError, match="wildcard") as e:
        eng.check_requests(persistence.request_columns(reqs[:5] + [(ns, "", r, s)]))
    assert e.value.code == L.EINVAL
    np.testing.assert_array_equal(eng.check_requests(persistence.request_columns(reqs)),
                                  _want(namespaces, rows, reqs))


@pytest.mark.gpu
@pytest.mark.parametrize("loop_self", [False, True])
def test_partition_device_rccl_world1_matches_oracle(loop_self, monkeypatch):
    """the native round over a real RCCL communicator of one rank (counts and bits through
    ncclAllGather; the records' own segment a copy-engine DMA, or with
    KETOGPU_TEST_RCCL_SELF=1 a grouped ncclSend/ncclRecv to the rank itself), the id exchange
    and request resolution over it too, every answer against the oracle"""
    if loop_self:
        monkeypatch.setenv("KETOGPU_TEST_RCCL_SELF", "1")
    from keto_amd import synth
    from keto_amd.partition import NativeComm, PartitionedEngine, Shard
    if L.lib().ketogpu_device_count() < 1:
        pytest.fail("no HIP device visible")
    w = synth.config5(users=50000, groups=5000, docs=20000, tuples=400_000, checks=12000, seed=29)
    from oracle import oracle as O
    st = O.Store(w.namespaces, 100)
    for cols in w.batches(1 << 16):
        st.add_columnar(cols)
    want = st.finalize(presorted=True).check_batch(w.requests(range(w.n_checks)), nthreads=8).astype(bool)
    comm = NativeComm(device=0, kind="rccl")
    sh = Shard.load(w.namespaces, lambda: w.batches(1 << 16), native_comm=comm)
    roots, targets, status = sh.resolve_batch(w.request_batch(), comm)
    assert not status.any()
    for direction in ("forward", "backward", "auto"):
        eng = PartitionedEngine(sh, device=0, direction=direction, comm=comm, record_capacity=1 << 20)
        np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
        st = eng.stats()
        assert st["collectives"] > 2 * st["levels"] and st["records_sent"] == st["records_received"] > 0
    # small buffers: overflowing rounds are retried with fewer requests over RCCL too
    eng = PartitionedEngine(sh, device=0, direction="backward", comm=comm, record_capacity=4096)
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
    assert eng.retries > 0
    cs = comm.stats()
    assert cs["rccl"] == 1 and cs["allgathers"] > 0
    assert (cs["sends"] > 0 and cs["recvs"] == cs["sends"]) if loop_self else cs["sends"] == 0
